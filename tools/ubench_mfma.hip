// f64 MFMA / VALU throughput microbenchmark (gfx950): cycles per
// v_mfma_f64_16x16x4_f64, per v_fma_f64, and both interleaved in one wave.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double v4d __attribute__((ext_vector_type(4)));

template <int MODE, int NCH>
__global__ __launch_bounds__(256, 1) void kernc(double *out, int iters)
{
    const int lane = threadIdx.x & 63;
    double a = 1.0 + lane * 1e-3, b = 0.5 - lane * 1e-4;
    v4d c[NCH];
#pragma unroll
    for (int i = 0; i < NCH; i++) c[i] = (v4d){0, 0, 0, 0};
    const unsigned long long t0 = __builtin_readcyclecounter();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NCH; i++) c[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[i], 0, 0, 0);
    }
    const unsigned long long t1 = __builtin_readcyclecounter();
    double s = 0;
#pragma unroll
    for (int i = 0; i < NCH; i++) s += c[i][0];
    if (lane == 0) out[blockIdx.x * 4 + (threadIdx.x >> 6)] = (double)(t1 - t0) / (iters * NCH);
    if (s == -12345.0) out[0] = s;
}

template <int MODE>
__global__ __launch_bounds__(256, 1) void kern(double *out, int iters)
{
    const int lane = threadIdx.x & 63;
    double a = 1.0 + lane * 1e-3, b = 0.5 - lane * 1e-4;
    v4d c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    double f[16];
#pragma unroll
    for (int i = 0; i < 16; i++) f[i] = lane + i;
    const unsigned long long t0 = __builtin_readcyclecounter();
    for (int it = 0; it < iters; ++it) {
        if constexpr (MODE == 0 || MODE == 2) {
            c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, a, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, b, c3, 0, 0, 0);
        }
        if constexpr (MODE == 1 || MODE == 2) {
#pragma unroll
            for (int r = 0; r < 2; r++)
#pragma unroll
                for (int i = 0; i < 16; i++) f[i] = fma(f[i], a, b);
        }
    }
    const unsigned long long t1 = __builtin_readcyclecounter();
    double s = c0[0] + c1[1] + c2[2] + c3[3];
#pragma unroll
    for (int i = 0; i < 16; i++) s += f[i];
    if (lane == 0) out[blockIdx.x * 4 + (threadIdx.x >> 6)] = (double)(t1 - t0) / iters;
    if (s == -12345.0) out[0] = s;
}

int main()
{
    const int blocks = 256, iters = 20000;   // one 4-wave block per CU: one wave per SIMD
    double *d;
    (void)hipMalloc(&d, blocks * 4 * sizeof(double));
    double *h = new double[blocks * 4];
    const char *names[3] = {"4 x mfma_f64_16x16x4 / iter", "32 x v_fma_f64 / iter", "both interleaved"};
    for (int m = 0; m < 3; m++) {
        hipEvent_t e0, e1;
        (void)hipEventCreate(&e0);
        (void)hipEventCreate(&e1);
        float ms = 0;
        for (int rep = 0; rep < 2; rep++) {
            (void)hipEventRecord(e0);
            if (m == 0) hipLaunchKernelGGL(kern<0>, dim3(blocks), dim3(256), 0, 0, d, iters);
            if (m == 1) hipLaunchKernelGGL(kern<1>, dim3(blocks), dim3(256), 0, 0, d, iters);
            if (m == 2) hipLaunchKernelGGL(kern<2>, dim3(blocks), dim3(256), 0, 0, d, iters);
            (void)hipEventRecord(e1);
            (void)hipEventSynchronize(e1);
            (void)hipEventElapsedTime(&ms, e0, e1);
        }
        (void)hipMemcpy(h, d, blocks * 4 * sizeof(double), hipMemcpyDeviceToHost);
        double s = 0;
        for (int i = 0; i < blocks * 4; i++) s += h[i];
        const double cyc = s / (blocks * 4);
        const double flops = (m != 1 ? 4.0 * 2048 * 64 / 64 : 0) + (m != 0 ? 32.0 * 2 * 64 : 0);  // per wave per iter
        const double tf = flops * iters * blocks * 4 / (ms * 1e-3) / 1e12;
        printf("%-30s %7.1f cycles/iter (readcyclecounter)  wall %.3f ms  %.1f TFLOP/s chip\n", names[m], cyc, ms, tf);
    }
    // chains: cycles per MFMA at 1 wave/SIMD (blocks=256) and 2 waves/SIMD (blocks=512)
    for (int nb : {256, 512}) {
        double *d2; (void)hipMalloc(&d2, nb * 4 * sizeof(double));
        double *h2 = new double[nb * 4];
        for (int ch : {1, 4, 8, 16}) {
            hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1); float ms = 0;
            for (int rep = 0; rep < 2; rep++) {
                (void)hipEventRecord(e0);
                if (ch == 1) hipLaunchKernelGGL((kernc<0, 1>), dim3(nb), dim3(256), 0, 0, d2, iters);
                if (ch == 4) hipLaunchKernelGGL((kernc<0, 4>), dim3(nb), dim3(256), 0, 0, d2, iters / 4);
                if (ch == 8) hipLaunchKernelGGL((kernc<0, 8>), dim3(nb), dim3(256), 0, 0, d2, iters / 8);
                if (ch == 16) hipLaunchKernelGGL((kernc<0, 16>), dim3(nb), dim3(256), 0, 0, d2, iters / 16);
                (void)hipEventRecord(e1); (void)hipEventSynchronize(e1); (void)hipEventElapsedTime(&ms, e0, e1);
            }
            (void)hipMemcpy(h2, d2, nb * 4 * sizeof(double), hipMemcpyDeviceToHost);
            double s = 0; for (int i = 0; i < nb * 4; i++) s += h2[i];
            const double tf = 2048.0 * iters * nb * 4 / (ms * 1e-3) / 1e12;
            printf("waves/SIMD %d chains %2d: %6.1f cycles per mfma_f64 (per wave)  %.1f TFLOP/s chip\n", nb / 256, ch, s / (nb * 4), tf);
        }
    }
    return 0;
}
