// ubench_dpp64.hip -- issue rate of v_fmac_f64 with a DPP row_newbcast source
// against the plain VOP2 form, 16 independent accumulators per lane, 3 waves
// per SIMD (the solve kernels' occupancy), all 256 CUs.  Decides whether the
// headline's in-panel operands are cheaper as DPP broadcasts than as LDS reads.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ __launch_bounds__(256) void kern(double *out, int iters, double a)
{
    double f[16];
#pragma unroll
    for (int i = 0; i < 16; i++) f[i] = threadIdx.x * 1e-9 + i;
    double src = a + threadIdx.x * 1e-12;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; i++) {
            if constexpr (MODE == 0)
                asm volatile("v_fmac_f64_e32 %0, %1, %2" : "+v"(f[i]) : "v"(src), "v"(f[(i + 1) & 15]));
            else if constexpr (MODE == 1)
                asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf"
                             : "+v"(f[i]) : "v"(src), "v"(f[(i + 1) & 15]));
            else   // VOP3 form with a negated operand (what the product's cmsub_conj emits)
                asm volatile("v_fma_f64 %0, -%1, %2, %0" : "+v"(f[i]) : "v"(src), "v"(f[(i + 1) & 15]));
        }
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) s += f[i];
    if (s == -12345.0) out[0] = s;
}

int main()
{
    double *d;
    (void)hipMalloc(&d, 64);
    const int iters = 2000, nb = 256 * 3;
    const char *names[3] = {"v_fmac_f64_e32", "v_fmac_f64_dpp row_newbcast", "v_fma_f64 (VOP3, neg)"};
    for (int mode = 0; mode < 3; ++mode) {
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        float best = 1e9;
        for (int rep = 0; rep < 5; rep++) {
            float ms = 0;
            (void)hipEventRecord(e0);
            if (mode == 0) hipLaunchKernelGGL(kern<0>, dim3(nb), dim3(256), 0, 0, d, iters, 0.999);
            else if (mode == 1) hipLaunchKernelGGL(kern<1>, dim3(nb), dim3(256), 0, 0, d, iters, 0.999);
            else hipLaunchKernelGGL(kern<2>, dim3(nb), dim3(256), 0, 0, d, iters, 0.999);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            (void)hipEventElapsedTime(&ms, e0, e1);
            if (rep && ms < best) best = ms;
        }
        const double wave_instrs = (double)iters * 16 * (nb * 4);          // per chip
        const double per_simd = wave_instrs / 1024.0;
        printf("%-30s %7.3f ms  %.2f ns per wave-instruction per SIMD  (%.1f TFLOP/s chip)\n", names[mode], best,
               best * 1e6 / per_simd, 2 * wave_instrs * 64 / (best * 1e-3) / 1e12);
    }
    return 0;
}
