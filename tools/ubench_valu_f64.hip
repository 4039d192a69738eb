// ubench_valu_f64.hip -- chip-wide v_fma_f64 issue rate against occupancy:
// 16 independent FMA chains per lane, 1..8 waves per SIMD (blocks of 4 waves,
// 256 CUs).  Settles the practical FP64 VALU ceiling the headline solve
// kernel (VALU-only, 3 waves/SIMD) is measured against.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int CH>
__global__ __launch_bounds__(256) void kern(double *out, int iters, double a, double b)
{
    double f[CH];
#pragma unroll
    for (int i = 0; i < CH; i++) f[i] = threadIdx.x * 1e-9 + i;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 4; r++)
#pragma unroll
            for (int i = 0; i < CH; i++) f[i] = fma(f[i], a, b);
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < CH; i++) s += f[i];
    if (s == -12345.0) out[0] = s;
}

int main()
{
    double *d;
    (void)hipMalloc(&d, 64);
    const int iters = 4000;
    for (int ch : {8, 16}) {
        for (int w : {1, 2, 3, 4, 8}) {
            const int nb = 256 * w;
            hipEvent_t e0, e1;
            (void)hipEventCreate(&e0);
            (void)hipEventCreate(&e1);
            float ms = 0;
            for (int rep = 0; rep < 3; rep++) {
                (void)hipEventRecord(e0);
                if (ch == 8) hipLaunchKernelGGL(kern<8>, dim3(nb), dim3(256), 0, 0, d, iters, 0.999, 1e-3);
                else hipLaunchKernelGGL(kern<16>, dim3(nb), dim3(256), 0, 0, d, iters, 0.999, 1e-3);
                (void)hipEventRecord(e1);
                (void)hipEventSynchronize(e1);
                (void)hipEventElapsedTime(&ms, e0, e1);
            }
            const double fmas = (double)iters * 4 * ch * 256.0 * nb;   // lane FMAs
            const double tf = 2 * fmas / (ms * 1e-3) / 1e12;
            printf("chains %2d  waves/SIMD %d: %7.3f ms  %5.1f TFLOP/s chip  (%.1f%% of 78.6)\n", ch, w, ms, tf,
                   100 * tf / 78.6);
        }
    }
    return 0;
}
