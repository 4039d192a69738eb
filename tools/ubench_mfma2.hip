// ubench_mfma2.hip -- FP64 pipe ceilings on gfx950, wall-clock timed
// (profiles/r02_ubench_mfma2.txt):
//   mfma  : v_mfma_f64_16x16x4_f64, NCH independent accumulators per wave
//   valu  : v_fma_f64, 16 independent chains per lane
//   mixed : in every workgroup, waves 0..M-1 run the MFMA loop and the rest
//           the VALU loop -- do the matrix and vector pipes of one SIMD
//           overlap when the instructions come from different waves?
// waves/SIMD = workgroups per CU (256 threads = one wave per SIMD each).
// build: hipcc -O3 --offload-arch=gfx950 tools/ubench_mfma2.hip -o tools/ubench_mfma2
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double v4d __attribute__((ext_vector_type(4)));

template <int NCH>
__device__ __forceinline__ double mfma_loop(int iters, double a, double b)
{
    v4d c[NCH];
#pragma unroll
    for (int i = 0; i < NCH; i++) c[i] = (v4d){0, 0, 0, 0};
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NCH; i++) c[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c[i], 0, 0, 0);
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < NCH; i++) s += c[i][0] + c[i][3];
    return s;
}
__device__ __forceinline__ double valu_loop(int iters, double a, double b, int lane)
{
    double f[16];
#pragma unroll
    for (int i = 0; i < 16; i++) f[i] = lane + i;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < 16; i++) f[i] = fma(f[i], a, b);
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) s += f[i];
    return s;
}

// mode 0: all MFMA; 1: all VALU; 2: wave w < nm MFMA, else VALU (waves of a
// 256-thread workgroup sit on different SIMDs); 3: 512-thread workgroups,
// waves 0..3 MFMA and 4..7 VALU -- waves w and w + 4 share SIMD w, so each
// SIMD holds one MFMA wave and one VALU wave
template <int NCH>
__global__ __launch_bounds__(512) void kern(double *out, int mode, int nm, int it_m, int it_v)
{
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const double a = 1.0 + lane * 1e-9, b = 1e-9 - lane * 1e-12;
    double s;
    const bool m = mode == 0 || (mode == 2 && w < nm) || (mode == 3 && w < 4);
    if (m) s = mfma_loop<NCH>(it_m, a, b);
    else s = valu_loop(it_v, a, b, lane);
    if (s == -12345.0) out[0] = s;
}

int main()
{
    double *out;
    hipMalloc(&out, 1024);
    int dev = 0, cus = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int it_m = 4000, it_v = 16000;
    auto run = [&](const char *name, int nch, int mode, int nm, int wps) {
        const int grid = cus * wps;
        auto launch = [&] {
            if (nch == 1) hipLaunchKernelGGL(kern<1>, dim3(grid), dim3(256), 0, 0, out, mode, nm, it_m, it_v);
            if (nch == 2) hipLaunchKernelGGL(kern<2>, dim3(grid), dim3(256), 0, 0, out, mode, nm, it_m, it_v);
            if (nch == 4) hipLaunchKernelGGL(kern<4>, dim3(grid), dim3(256), 0, 0, out, mode, nm, it_m, it_v);
            if (nch == 8) hipLaunchKernelGGL(kern<8>, dim3(grid), dim3(256), 0, 0, out, mode, nm, it_m, it_v);
        };
        launch();
        hipEventRecord(e0);
        for (int r = 0; r < 5; ++r) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        ms /= 5;
        // flops: MFMA waves nch * it_m * 2048; VALU waves 16 * it_v * 64 lanes * 2
        const double waves = (double)grid * 4;
        const double fm = mode == 0 ? waves : mode == 2 ? waves * nm / 4 : 0;
        const double fv = waves - fm;
        const double tf_m = fm * nch * (double)it_m * 2048 / (ms * 1e-3) / 1e12;
        const double tf_v = fv * 16.0 * it_v * 128 / (ms * 1e-3) / 1e12;
        printf("%-6s waves/SIMD %d nch %d mfma-waves/wg %d: %8.3f ms  mfma %5.1f TF  valu %5.1f TF  sum %5.1f TF\n",
               name, wps, nch, mode == 0 ? 4 : mode == 1 ? 0 : nm, ms, tf_m, tf_v, tf_m + tf_v);
    };
    for (int wps = 1; wps <= 4; ++wps)
        for (int nch : {1, 2, 4, 8}) run("mfma", nch, 0, 4, wps);
    for (int wps = 1; wps <= 4; ++wps) run("valu", 1, 1, 0, wps);
    for (int wps = 1; wps <= 4; ++wps)
        for (int nm : {1, 2}) run("mixed", 4, 2, nm, wps);
    // same-SIMD pairs: 512-thread workgroups
    auto run8 = [&](const char *name, int mode, int wgs) {
        const int grid = cus * wgs;
        auto launch = [&] { hipLaunchKernelGGL(kern<4>, dim3(grid), dim3(512), 0, 0, out, mode, 0, it_m, it_v); };
        launch();
        hipEventRecord(e0);
        for (int r = 0; r < 5; ++r) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        ms /= 5;
        const double waves = (double)grid * 8;
        const double fm = mode == 0 ? waves : mode == 3 ? waves / 2 : 0, fv = waves - fm;
        const double tf_m = fm * 4 * (double)it_m * 2048 / (ms * 1e-3) / 1e12;
        const double tf_v = fv * 16.0 * it_v * 128 / (ms * 1e-3) / 1e12;
        printf("%-10s wg512 x %d/CU (waves/SIMD %d): %8.3f ms  mfma %5.1f TF  valu %5.1f TF  sum %5.1f TF\n", name, wgs,
               2 * wgs, ms, tf_m, tf_v, tf_m + tf_v);
    };
    for (int wgs = 1; wgs <= 2; ++wgs) {
        run8("mfma-only", 0, wgs);
        run8("valu-only", 1, wgs);
        run8("same-simd", 3, wgs);
    }
    hipDeviceSynchronize();
    return 0;
}
