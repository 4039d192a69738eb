// ubench_mfma4.hip -- v_mfma_f64_4x4x4_4b_f64 on gfx950: operand/result lane
// layout (probed), throughput with independent accumulators, and the latency
// of a dependent chain (profiles/r02_ubench_mfma4.txt).
// build: hipcc -O3 --offload-arch=gfx950 tools/ubench_mfma4.hip -o tools/ubench_mfma4
#include <hip/hip_runtime.h>
#include <cstdio>

// probe: A one-hot at lane j, B[lane] = lane + 1 -> D[lane] = B value paired with A's (m, k)
__global__ void probe(double *out)
{
    const int l = threadIdx.x;
    for (int j = 0; j < 64; ++j) {
        const double a = (l == j) ? 1.0 : 0.0, b = l + 1.0;
        const double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
        out[j * 64 + l] = d;
    }
}

template <int NCH>
__global__ __launch_bounds__(512) void thr(double *out, int iters)
{
    const int lane = threadIdx.x & 63;
    const double a = 1.0 + lane * 1e-9, b = 1e-9 - lane * 1e-12;
    double c[NCH];
#pragma unroll
    for (int i = 0; i < NCH; i++) c[i] = 0;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int i = 0; i < NCH; i++) c[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c[i], 0, 0, 0);
    }
    double s = 0;
#pragma unroll
    for (int i = 0; i < NCH; i++) s += c[i];
    if (s == -12345.0) out[0] = s;
}

int main()
{
    double *d;
    hipMalloc(&d, 64 * 64 * 8);
    hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, d);
    double h[64 * 64];
    hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost);
    printf("probe: A one-hot at lane j -> output lanes L with D[L] = (B lane + 1)\n");
    for (int j = 0; j < 64; ++j) {
        printf("j=%2d:", j);
        for (int l = 0; l < 64; ++l)
            if (h[j * 64 + l] != 0) printf(" %d<-%d", l, (int)h[j * 64 + l] - 1);
        printf("\n");
    }
    int dev = 0, cus = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 20000;
    auto run = [&](int nch, int wps) {
        const int grid = cus * wps / 2;   // 512-thread workgroups: 2 waves per SIMD each
        auto launch = [&] {
            if (nch == 1) hipLaunchKernelGGL(thr<1>, dim3(grid), dim3(512), 0, 0, d, iters);
            if (nch == 2) hipLaunchKernelGGL(thr<2>, dim3(grid), dim3(512), 0, 0, d, iters);
            if (nch == 4) hipLaunchKernelGGL(thr<4>, dim3(grid), dim3(512), 0, 0, d, iters);
            if (nch == 8) hipLaunchKernelGGL(thr<8>, dim3(grid), dim3(512), 0, 0, d, iters);
        };
        launch();
        hipEventRecord(e0);
        for (int r = 0; r < 5; ++r) launch();
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        ms /= 5;
        const double waves = (double)grid * 8, inst = waves * nch * (double)iters;
        printf("4x4x4_4b: waves/SIMD %d chains %d: %8.3f ms  %6.1f TF  (%.1f ns per instr per wave-chain)\n", wps, nch,
               ms, inst * 512 / (ms * 1e-3) / 1e12, ms * 1e6 / ((double)iters * nch));
    };
    for (int wps : {2, 4})
        for (int nch : {1, 2, 4, 8}) run(nch, wps);
    hipDeviceSynchronize();
    return 0;
}
