// ubench_hbm.hip -- HBM ceilings of the access patterns the HBM-bound kernels
// combine (profiles/r02_ubench_hbm.txt).  1,048,576 frames of the bench's
// layouts: full frames (15 x 53 complex fp64, 12,720 B apart) for the pilot
// gathers, 53-element (848 B) rows for the streams.
//   write      : 848 B/frame streamed out, plain / nontemporal 16-B stores
//   read       : 848 B/frame streamed in (summed, one store per wave)
//   copy       : 848 B/frame in + 848 B out
//   gather     : the 8 pilot reads of a frame (4 tx + 4 rx, 16 B each, 64-B
//                sectors), one 16-B result per frame
//   gather+write: the REF kernel's traffic (8 pilot sectors + 848 B out)
// build: hipcc -O3 --offload-arch=gfx950 tools/ubench_hbm.hip -o tools/ubench_hbm
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

typedef double v2d __attribute__((ext_vector_type(2)));
constexpr int NSC = 53, FS = 795;
constexpr int P[4] = {5, 19, 33, 47};

template <bool NT>
__global__ __launch_bounds__(256) void k_write(v2d *o, int64_t n)
{
    const v2d v = {1.0, 2.0};
    for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        if (NT) __builtin_nontemporal_store(v, o + i);
        else o[i] = v;
    }
}
__global__ __launch_bounds__(256) void k_read(const v2d *in, v2d *o, int64_t n)
{
    v2d acc = {0, 0};
    for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) acc += in[i];
    if (acc.x == 12345.0) o[threadIdx.x] = acc;   // never true: keeps the loads
}
__global__ __launch_bounds__(256) void k_copy(const v2d *in, v2d *o, int64_t n)
{
    for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
        __builtin_nontemporal_store(in[i], o + i);
}
// one lane per frame: 8 pilot loads, one 16-B store
__global__ __launch_bounds__(256) void k_gather(const v2d *tx, const v2d *rx, v2d *o, int64_t nf)
{
    for (int64_t f = blockIdx.x * 256ll + threadIdx.x; f < nf; f += (int64_t)gridDim.x * 256) {
        v2d acc = {0, 0};
#pragma unroll
        for (int p = 0; p < 4; ++p) acc += tx[f * FS + P[p]] * rx[f * FS + P[p]];
        o[f] = acc;
    }
}
// gather + the 53-element output row per frame: a wave owns 64 frames
__global__ __launch_bounds__(256) void k_gather_write(const v2d *tx, const v2d *rx, v2d *o, int64_t nf)
{
    __shared__ v2d tab[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t ntile = (nf + 63) / 64;
    for (int64_t t = blockIdx.x * 4ll + w; t < ntile; t += (int64_t)gridDim.x * 4) {
        const int64_t f = t * 64 + lane;
        v2d acc = {0, 0};
        if (f < nf) {
#pragma unroll
            for (int p = 0; p < 4; ++p) acc += tx[f * FS + P[p]] * rx[f * FS + P[p]];
        }
        tab[w][lane] = acc;
        __builtin_amdgcn_wave_barrier();
        for (int i = 0; i < NSC; ++i) {
            const int e = 64 * i + lane, fl = e / NSC;
            __builtin_nontemporal_store(tab[w][fl], o + t * 64 * NSC + e);
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// one wave per contiguous run of `run` 16-B elements (the tile kernels' store pattern)
__global__ __launch_bounds__(256) void k_write_runs(v2d *o, int64_t n, int run)
{
    const v2d v = {1.0, 2.0};
    const int lane = threadIdx.x & 63;
    const int64_t nruns = (n + run - 1) / run;
    for (int64_t r = blockIdx.x * 4ll + (threadIdx.x >> 6); r < nruns; r += (int64_t)gridDim.x * 4)
        for (int i = lane; i < run; i += 64) {
            const int64_t e = r * run + i;
            if (e < n) __builtin_nontemporal_store(v, o + e);
        }
}
// LS (configs[1]) traffic without the arithmetic: per frame 848 B streamed in
// (rx_pre), the 8 pilot reads of a 53-element row (dense rows, 848 B apart),
// 2 x 848 B streamed out; a wave owns 64 frames
__global__ __launch_bounds__(256) void k_ls_like(const v2d *pre, const v2d *tx, const v2d *rx, v2d *o1, v2d *o2,
                                                 int64_t nf)
{
    __shared__ v2d tab[4][64];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t ntile = (nf + 63) / 64;
    for (int64_t t = blockIdx.x * 4ll + w; t < ntile; t += (int64_t)gridDim.x * 4) {
        const int64_t f = t * 64 + lane;
        v2d acc = {0, 0};
#pragma unroll
        for (int p = 0; p < 4; ++p) acc += tx[f * NSC + P[p]] * rx[f * NSC + P[p]];
        tab[w][lane] = acc;
        __builtin_amdgcn_wave_barrier();
#pragma unroll 4
        for (int i = 0; i < NSC; ++i) {
            const int64_t e = t * 64 * NSC + 64 * i + lane;
            const v2d x = pre[e] * tab[w][(64 * i + lane) / NSC];
            __builtin_nontemporal_store(x, o1 + e);
            __builtin_nontemporal_store(x + x, o2 + e);
        }
        __builtin_amdgcn_wave_barrier();
    }
}

// one element per thread, no grid stride: the pattern write_nt_1pt measured fastest
__global__ __launch_bounds__(256) void k_copy2_1pt(const v2d *in, const v2d *tab, v2d *o1, v2d *o2, int64_t n)
{
    const int64_t e = blockIdx.x * 256ll + threadIdx.x;
    if (e >= n) return;
    const v2d x = in[e] * tab[e / NSC];
    __builtin_nontemporal_store(x, o1 + e);
    __builtin_nontemporal_store(x + x, o2 + e);
}
__global__ __launch_bounds__(256) void k_write_tab_1pt(const v2d *tab, v2d *o, int64_t n)
{
    const int64_t e = blockIdx.x * 256ll + threadIdx.x;
    if (e >= n) return;
    __builtin_nontemporal_store(tab[e / NSC], o + e);
}
// dense-row pilot gather (LS layout: 53-element rows), one 16-B value per frame
__global__ __launch_bounds__(256) void k_gather_dense(const v2d *tx, const v2d *rx, v2d *o, int64_t nf)
{
    const int64_t f = blockIdx.x * 256ll + threadIdx.x;
    if (f >= nf) return;
    v2d acc = {0, 0};
#pragma unroll
    for (int p = 0; p < 4; ++p) acc += tx[f * NSC + P[p]] * rx[f * NSC + P[p]];
    o[f] = acc;
}

// wave-level phase separation: a wave gathers the pilots of FPW frames (FPW/64
// rounds of one frame per lane) before it writes any of their outputs; with
// every wave resident, the gathers of the whole batch come first
template <int FPW>
__global__ __launch_bounds__(256) void k_gather_write_big(const v2d *tx, const v2d *rx, v2d *o, int64_t nf)
{
    __shared__ v2d tab[4][FPW];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t ntile = (nf + FPW - 1) / FPW;
    for (int64_t t = blockIdx.x * 4ll + w; t < ntile; t += (int64_t)gridDim.x * 4) {
#pragma unroll
        for (int r = 0; r < FPW / 64; ++r) {
            const int64_t f = t * FPW + r * 64 + lane;
            v2d acc = {0, 0};
            if (f < nf) {
#pragma unroll
                for (int p = 0; p < 4; ++p) acc += tx[f * FS + P[p]] * rx[f * FS + P[p]];
            }
            tab[w][r * 64 + lane] = acc;
        }
        __builtin_amdgcn_wave_barrier();
        for (int i = lane; i < FPW * NSC; i += 64)
            __builtin_nontemporal_store(tab[w][i / NSC], o + t * FPW * NSC + i);
        __builtin_amdgcn_wave_barrier();
    }
}

int main(int argc, char **argv)
{
    const int64_t nf = 1 << 20;
    const int64_t nel = nf * NSC;
    v2d *tx, *rx, *a, *b;
    CK(hipMalloc(&tx, nf * FS * 16));
    CK(hipMalloc(&rx, nf * FS * 16));
    CK(hipMalloc(&a, nel * 16));
    CK(hipMalloc(&b, nel * 16));
    CK(hipMemset(tx, 0, nf * FS * 16));
    CK(hipMemset(rx, 0, nf * FS * 16));
    CK(hipMemset(a, 0, nel * 16));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int reps = 20;
    auto timeit = [&](const char *name, double bytes, auto launch) {
        for (int g : {1024, 2048, 4096, 8192, 16384}) {
            for (int i = 0; i < 3; ++i) launch(g);
            hipEventRecord(e0);
            for (int i = 0; i < reps; ++i) launch(g);
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            ms /= reps;
            printf("%-14s grid %5d: %8.1f us  %6.2f TB/s\n", name, g, ms * 1e3, bytes / (ms * 1e-3) / 1e12);
        }
    };
    timeit("write", nel * 16.0, [&](int g) { hipLaunchKernelGGL(k_write<false>, dim3(g), dim3(256), 0, 0, a, nel); });
    timeit("write_nt", nel * 16.0, [&](int g) { hipLaunchKernelGGL(k_write<true>, dim3(g), dim3(256), 0, 0, a, nel); });
    timeit("read", nel * 16.0, [&](int g) { hipLaunchKernelGGL(k_read, dim3(g), dim3(256), 0, 0, a, b, nel); });
    timeit("copy_nt", nel * 32.0, [&](int g) { hipLaunchKernelGGL(k_copy, dim3(g), dim3(256), 0, 0, a, b, nel); });
    timeit("gather(sect)", nf * (8 * 64.0 + 16), [&](int g) { hipLaunchKernelGGL(k_gather, dim3(g), dim3(256), 0, 0, tx, rx, b, nf); });
    timeit("gather+write", nf * (8 * 64.0 + 848), [&](int g) { hipLaunchKernelGGL(k_gather_write, dim3(g), dim3(256), 0, 0, tx, rx, b, nf); });
    {   // writes: one element per thread (no grid stride), and per-wave contiguous runs
        const int64_t g = (nel + 255) / 256;
        for (int i = 0; i < 3; ++i) hipLaunchKernelGGL(k_write<true>, dim3(g), dim3(256), 0, 0, a, nel);
        hipEventRecord(e0);
        for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k_write<true>, dim3(g), dim3(256), 0, 0, a, nel);
        hipEventRecord(e1);
        hipEventSynchronize(e1);
        float ms;
        hipEventElapsedTime(&ms, e0, e1);
        ms /= reps;
        printf("%-14s grid %5lld: %8.1f us  %6.2f TB/s\n", "write_nt_1pt", (long long)g, ms * 1e3, nel * 16.0 / (ms * 1e-3) / 1e12);
    }
    for (int run : {3392, 16384, 65536})
        timeit(run == 3392 ? "write_run54K" : run == 16384 ? "write_run256K" : "write_run1M", nel * 16.0,
               [&](int g) { hipLaunchKernelGGL(k_write_runs, dim3(g), dim3(256), 0, 0, a, nel, run); });
    {
        v2d *pre, *t2, *r2, *o2;
        CK(hipMalloc(&pre, nel * 16));
        CK(hipMalloc(&t2, nel * 16));
        CK(hipMalloc(&r2, nel * 16));
        CK(hipMalloc(&o2, nel * 16));
        CK(hipMemset(pre, 0, nel * 16));
        CK(hipMemset(t2, 0, nel * 16));
        CK(hipMemset(r2, 0, nel * 16));
        timeit("ls_like(alg)", nf * 2672.0,
               [&](int g) { hipLaunchKernelGGL(k_ls_like, dim3(g), dim3(256), 0, 0, pre, t2, r2, a, o2, nf); });
    }
    {
        v2d *pre, *t2, *r2, *o2, *tab;
        CK(hipMalloc(&pre, nel * 16));
        CK(hipMalloc(&t2, nel * 16));
        CK(hipMalloc(&r2, nel * 16));
        CK(hipMalloc(&o2, nel * 16));
        CK(hipMalloc(&tab, nf * 16));
        CK(hipMemset(pre, 0, nel * 16));
        CK(hipMemset(t2, 0, nel * 16));
        CK(hipMemset(r2, 0, nel * 16));
        CK(hipMemset(tab, 0, nf * 16));
        const int64_t ge = (nel + 255) / 256, gf = (nf + 255) / 256;
        auto one = [&](const char *name, double bytes, auto launch) {
            for (int i = 0; i < 3; ++i) launch();
            hipEventRecord(e0);
            for (int i = 0; i < reps; ++i) launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            ms /= reps;
            printf("%-22s: %8.1f us  %6.2f TB/s\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e12);
        };
        // REF in two phases: full-frame pilot gather -> 16 B/frame, then one-shot writes
        one("ref2:gather(sect)", nf * (8 * 64.0 + 16), [&] { hipLaunchKernelGGL(k_gather, dim3(gf), dim3(256), 0, 0, tx, rx, tab, nf); });
        one("ref2:write_1pt", nel * 16.0, [&] { hipLaunchKernelGGL(k_write_tab_1pt, dim3(ge), dim3(256), 0, 0, tab, a, nel); });
        one("ref2:both(sect)", nf * (8 * 64.0 + 848), [&] {
            hipLaunchKernelGGL(k_gather, dim3(gf), dim3(256), 0, 0, tx, rx, tab, nf);
            hipLaunchKernelGGL(k_write_tab_1pt, dim3(ge), dim3(256), 0, 0, tab, a, nel);
        });
        for (int fpw : {128, 256, 512}) {
            const int64_t g = (nf / fpw + 3) / 4;
            char name[64];
            snprintf(name, sizeof name, "ref:big%d(sect)", fpw);
            one(name, nf * (8 * 64.0 + 848), [&] {
                if (fpw == 128) hipLaunchKernelGGL(k_gather_write_big<128>, dim3(g), dim3(256), 0, 0, tx, rx, a, nf);
                if (fpw == 256) hipLaunchKernelGGL(k_gather_write_big<256>, dim3(g), dim3(256), 0, 0, tx, rx, a, nf);
                if (fpw == 512) hipLaunchKernelGGL(k_gather_write_big<512>, dim3(g), dim3(256), 0, 0, tx, rx, a, nf);
            });
        }
        // LS in two phases: dense-row pilot gather, then one-shot stream (848 in, 2 x 848 out)
        one("ls2:gather_dense", nf * 8 * 64.0, [&] { hipLaunchKernelGGL(k_gather_dense, dim3(gf), dim3(256), 0, 0, t2, r2, tab, nf); });
        one("ls2:copy2_1pt", nel * 48.0, [&] { hipLaunchKernelGGL(k_copy2_1pt, dim3(ge), dim3(256), 0, 0, pre, tab, a, o2, nel); });
        one("ls2:both(alg)", nf * 2672.0, [&] {
            hipLaunchKernelGGL(k_gather_dense, dim3(gf), dim3(256), 0, 0, t2, r2, tab, nf);
            hipLaunchKernelGGL(k_copy2_1pt, dim3(ge), dim3(256), 0, 0, pre, tab, a, o2, nel);
        });
    }
    CK(hipDeviceSynchronize());
    printf("(gather rates count 64 B per pilot read: the sector floor)\n");
    return 0;
}
