// LDS microbenchmark (gfx950): cycles per wave-instruction, 12 waves/CU, for
// the access shapes the MMSE solve uses.  hipcc -O3 --offload-arch=gfx950.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ __launch_bounds__(64, 3) void kern(double *out, int iters)
{
    __shared__ double2 buf[2][64];
    const int lane = threadIdx.x, p = lane >> 3, q = lane & 7;
    double2 acc = make_double2(lane, 0), v = make_double2(1.0 + lane, 2.0);
    buf[0][lane] = v;
    buf[1][lane] = v;
    __syncthreads();
    const unsigned long long t0 = __builtin_readcyclecounter();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 7; ++r) {
            if constexpr (MODE == 0) {          // masked write: 8 active lanes (q == kq)
                if (q == (it & 7)) buf[it & 1][p + 8 * r] = v;
            } else if constexpr (MODE == 1) {   // full write: 64 lanes
                buf[it & 1][(lane + r) & 63] = v;
            } else if constexpr (MODE == 4) {   // masked write, 8 lanes, two b64 halves
                if (q == (it & 7)) {
                    double *d = reinterpret_cast<double *>(&buf[it & 1][p + 8 * r]);
                    d[0] = v.x;
                    d[1] = v.y;
                }
            } else if constexpr (MODE == 5) {   // masked write, 8 lanes, b64 (re only)
                if (q == (it & 7)) reinterpret_cast<double *>(&buf[it & 1][p + 8 * r])[0] = v.x;
            } else if constexpr (MODE == 6) {   // masked write, 8 lanes, b32
                if (q == (it & 7)) reinterpret_cast<float *>(&buf[it & 1][p + 8 * r])[0] = (float)v.x;
            } else if constexpr (MODE == 2) {   // broadcast read, 8 distinct addresses
                double2 t = buf[it & 1][p + 8 * r];
                acc.x += t.x; acc.y += t.y;
            } else {                            // read, 64 distinct addresses
                double2 t = buf[it & 1][(lane + r) & 63];
                acc.x += t.x; acc.y += t.y;
            }
        }
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        v.x += 1.0;
    }
    const unsigned long long t1 = __builtin_readcyclecounter();
    if (lane == 0) out[blockIdx.x] = (double)(t1 - t0) / (iters * 7.0);
    if (acc.x == -1.0) out[0] = acc.y;
}

int main()
{
    const int blocks = 256 * 12, iters = 2000;
    double *d;
    (void)hipMalloc(&d, blocks * sizeof(double));
    double *h = new double[blocks];
    const char *names[7] = {"ds_write_b128 8 lanes", "ds_write_b128 64 lanes", "ds_read_b128 bcast(8 addr)",
                            "ds_read_b128 64 addr", "2x ds_write_b64 8 lanes", "ds_write_b64 8 lanes",
                            "ds_write_b32 8 lanes"};
    for (int m = 0; m < 7; m++) {
        hipEvent_t a, b;
        (void)hipEventCreate(&a);
        (void)hipEventCreate(&b);
        for (int rep = 0; rep < 2; rep++) {
            (void)hipEventRecord(a);
            if (m == 0) hipLaunchKernelGGL(kern<0>, dim3(blocks), dim3(64), 0, 0, d, iters);
            if (m == 1) hipLaunchKernelGGL(kern<1>, dim3(blocks), dim3(64), 0, 0, d, iters);
            if (m == 2) hipLaunchKernelGGL(kern<2>, dim3(blocks), dim3(64), 0, 0, d, iters);
            if (m == 3) hipLaunchKernelGGL(kern<3>, dim3(blocks), dim3(64), 0, 0, d, iters);
            if (m == 4) hipLaunchKernelGGL(kern<4>, dim3(blocks), dim3(64), 0, 0, d, iters);
            if (m == 5) hipLaunchKernelGGL(kern<5>, dim3(blocks), dim3(64), 0, 0, d, iters);
            if (m == 6) hipLaunchKernelGGL(kern<6>, dim3(blocks), dim3(64), 0, 0, d, iters);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
        }
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        (void)hipMemcpy(h, d, blocks * sizeof(double), hipMemcpyDeviceToHost);
        double s = 0;
        for (int i = 0; i < blocks; i++) s += h[i];
        // per-CU cost: 12 waves share one LDS; wall ms -> cycles at measured rate
        const double instr_per_cu = 12.0 * iters * 7.0;
        printf("%-28s wave-view %.1f cyc/instr   CU throughput %.2f ns/instr (%.2f cyc @2.1GHz)\n", names[m],
               s / blocks, ms * 1e6 / instr_per_cu, ms * 1e6 / instr_per_cu * 2.1);
    }
    return 0;
}
