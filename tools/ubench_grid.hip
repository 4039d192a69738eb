// ubench_grid.hip -- the headline solve's trailing update on the two lane
// grids of round-2 review item 5, measured instead of modelled
// (tools/grid_model.py counts issues; this times them).
//
// One wave per frame, 3 waves/SIMD (the product kernel's occupancy), 65,536
// frames.  Per pivot step k = 1..52 (the product's pivots after the exact
// first step), with trailing columns j >= 8 (k / 8) + 8 as the row-panel
// Cholesky leaves them:
//   publish   every lane stores one complex of column c_k to LDS (the value
//             depends on the previous step's update, as the pivot chain does)
//   operands  8x8 grid: one ds_read_b128 per live block row (c[p + 8 aa]) and
//             per live block column (c[q + 8 bb]);
//             4x16 grid: ONE ds_read_b128 of row operands (lane 16 p + a holds
//             c[p + 4 a]) handed out by v_fmac_f64_dpp row_newbcast:a, plus
//             one read per live 16-wide block column (c[q + 16 b])
//   update    A[blk] -= c_i conj(c_j): 4 FP64 FMAs per live register block.
// The 8x8 grid holds 28 lower blocks (112 VGPRs), the 4x16 grid 32 (128).
// Everything else in the product kernel (the panels, the pivot chain, the
// build, the read-out) is the same for both grids and left out.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

constexpr int NR = 55, NCOL = 53, NF = 65536;

__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    __builtin_amdgcn_sched_barrier(0);   // steps stay in order: one straight-line block otherwise
}

// live: register block rows [r0, r0 + bh) x columns [c0, c0 + bw) hold an
// element i >= j with j >= jmin, i < NR, j < NCOL
__host__ __device__ constexpr bool live(int r0, int bh, int c0, int bw, int jmin)
{
    for (int i = r0; i < r0 + bh && i < NR; ++i)
        for (int j = c0; j < c0 + bw && j < NCOL; ++j)
            if (i >= j && j >= jmin) return true;
    return false;
}
__host__ __device__ constexpr bool stored(int r0, int bh, int c0, int bw) { return live(r0, bh, c0, bw, 0); }

// acc -= r conj(c), issued here: the empty volatile asm keeps the compiler from
// sinking the update chains towards the final checksum (the product kernel's
// pivot chain consumes every update in the step it is made)
__device__ __forceinline__ void csub_conj(double2 &acc, double2 r, double2 c)
{
    acc.x = fma(-r.x, c.x, fma(-r.y, c.y, acc.x));
    acc.y = fma(-r.y, c.x, fma(r.x, c.y, acc.y));
    asm volatile("" : "+v"(acc.x), "+v"(acc.y));
}

// ---- 8x8 grid: lane (p, q) = (lane >> 3, lane & 7), block (aa, bb) holds A[p + 8 aa][q + 8 bb]
// column operand of block column B0 read once, then every live block (A0 >= B0) of that column
template <int A0, int B0, int JM>
__device__ __forceinline__ void upd8col(double2 (&A)[7][7], const double2 (&ur)[7], double2 c)
{
    if constexpr (A0 < 7) {
        if constexpr (live(8 * A0, 8, 8 * B0, 8, JM)) csub_conj(A[A0][B0], ur[A0], c);
        upd8col<A0 + 1, B0, JM>(A, ur, c);
    }
}
template <int B0, int JM>
__device__ __forceinline__ void upd8(double2 (&A)[7][7], const double2 (&ur)[7], const double2 *col, int q)
{
    if constexpr (B0 < 7) {
        if constexpr (live(8 * B0, 56 - 8 * B0, 8 * B0, 8, JM)) upd8col<B0, B0, JM>(A, ur, col[q + 8 * B0]);
        upd8<B0 + 1, JM>(A, ur, col, q);
    }
}
// panel KB: pivots k = 8 KB .. 8 KB + 7 (from 1, below 53), trailing columns j >= 8 KB + 8
template <int KB>
__device__ __forceinline__ void panel8(double2 (&A)[7][7], double2 *col, int p, int q, int lane)
{
    if constexpr (KB < 7) {
        constexpr int JM = 8 * KB + 8;
#pragma unroll
        for (int kq = 0; kq < 8; ++kq) {
            const int k = 8 * KB + kq;
            if (k == 0 || k >= NCOL) continue;
            // publish: depends on the last step's update
            col[lane] = make_double2(A[6][KB < 6 ? KB + 1 : 6].x * 1e-3 + lane, A[6][KB < 6 ? KB + 1 : 6].y * 1e-3);
            wave_sync();
            double2 ur[7];
#pragma unroll
            for (int a = 0; a < 7; ++a) ur[a] = a > KB ? col[p + 8 * a] : make_double2(0.0, 0.0);
            if constexpr (JM < NCOL) upd8<0, JM>(A, ur, col, q);
            wave_sync();
        }
        panel8<KB + 1>(A, col, p, q, lane);
    }
}

__global__ __launch_bounds__(64, 3) void grid8_kernel(double *out)
{
    __shared__ double2 col[64];
    const int lane = threadIdx.x, p = lane >> 3, q = lane & 7;
    double2 A[7][7];
#pragma unroll
    for (int a = 0; a < 7; ++a)
#pragma unroll
        for (int b = 0; b <= a; ++b) A[a][b] = make_double2(1.0 + 1e-3 * (a * 7 + b + lane), 1e-4 * lane);
    panel8<0>(A, col, p, q, lane);
    double s = 0;
#pragma unroll
    for (int a = 0; a < 7; ++a)
#pragma unroll
        for (int b = 0; b <= a; ++b) s += A[a][b].x + A[a][b].y;
    out[(size_t)blockIdx.x * 64 + lane] = s;
}

// ---- 4x16 grid: lane (p, q) = (lane >> 4, lane & 15), block (a, b) holds A[p + 4 a][q + 16 b]
// acc -= R[lane 16 p + N] conj(c): the row operand by row_newbcast:N (the register comes
// straight from a ds_read, so no VALU-write-to-DPP-read hazard can arise)
template <int N>
__device__ __forceinline__ void csub_conj_bc(double2 &acc, double2 R, double2 c)
{
    asm volatile("v_fmac_f64_dpp %[ax], -%[rx], %[cx] row_newbcast:%c[n] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %[ax], -%[ry], %[cy] row_newbcast:%c[n] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %[ay], -%[ry], %[cx] row_newbcast:%c[n] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %[ay], %[rx], %[cy] row_newbcast:%c[n] row_mask:0xf bank_mask:0xf"
        : [ax] "+v"(acc.x), [ay] "+v"(acc.y)
        : [rx] "v"(R.x), [ry] "v"(R.y), [cx] "v"(c.x), [cy] "v"(c.y), [n] "i"(N));
}

template <int A0, int B0, int JM>
__device__ __forceinline__ void upd16(double2 (&A)[14][4], double2 R, const double2 (&cc)[4])
{
    if constexpr (A0 < 14) {
        if constexpr (B0 < 4) {
            if constexpr (stored(4 * A0, 4, 16 * B0, 16) && live(4 * A0, 4, 16 * B0, 16, JM))
                csub_conj_bc<A0>(A[A0][B0], R, cc[B0]);
            upd16<A0, B0 + 1, JM>(A, R, cc);
        } else {
            upd16<A0 + 1, 0, JM>(A, R, cc);
        }
    }
}

template <int KB>
__device__ __forceinline__ void panel16(double2 (&A)[14][4], double2 *col, int p, int q, int lane)
{
    if constexpr (KB < 7) {
        constexpr int JM = 8 * KB + 8;
        constexpr int BL = JM / 16;   // first live block column
#pragma unroll
        for (int kq = 0; kq < 8; ++kq) {
            const int k = 8 * KB + kq;
            if (k == 0 || k >= NCOL) continue;
            col[lane] = make_double2(A[13][BL < 4 ? BL : 3].x * 1e-3 + lane, A[13][BL < 4 ? BL : 3].y * 1e-3);
            wave_sync();
            const double2 R = col[p + 4 * (q < 14 ? q : 13)];   // row operands of all 14 block rows, one read
            double2 cc[4];
#pragma unroll
            for (int b = 0; b < 4; ++b)
                cc[b] = b >= BL && JM < NCOL ? col[q + 16 * b < 64 ? q + 16 * b : 63] : make_double2(0.0, 0.0);
            if constexpr (JM < NCOL) upd16<0, 0, JM>(A, R, cc);
            wave_sync();
        }
        panel16<KB + 1>(A, col, p, q, lane);
    }
}

__global__ __launch_bounds__(64, 3) void grid16_kernel(double *out)
{
    __shared__ double2 col[64];
    const int lane = threadIdx.x, p = lane >> 4, q = lane & 15;
    double2 A[14][4];
#pragma unroll
    for (int a = 0; a < 14; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
            A[a][b] = stored(4 * a, 4, 16 * b, 16) ? make_double2(1.0 + 1e-3 * (a * 4 + b + lane), 1e-4 * lane)
                                                   : make_double2(0.0, 0.0);
    panel16<0>(A, col, p, q, lane);
    double s = 0;
#pragma unroll
    for (int a = 0; a < 14; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
            if (stored(4 * a, 4, 16 * b, 16)) s += A[a][b].x + A[a][b].y;
    out[(size_t)blockIdx.x * 64 + lane] = s;
}

int main(int argc, char **argv)
{
    const int rounds = argc > 1 ? atoi(argv[1]) : 7, reps = 20;
    double *d;
    if (hipMalloc(&d, (size_t)NF * 64 * sizeof(double)) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    float best[2] = {1e30f, 1e30f}, med[2][64];
    for (int r = 0; r < rounds; ++r)
        for (int g = 0; g < 2; ++g) {
            for (int w = 0; w < 3; ++w) {
                if (g == 0) hipLaunchKernelGGL(grid8_kernel, dim3(NF), dim3(64), 0, 0, d);
                else hipLaunchKernelGGL(grid16_kernel, dim3(NF), dim3(64), 0, 0, d);
            }
            (void)hipEventRecord(e0, 0);
            for (int i = 0; i < reps; ++i) {
                if (g == 0) hipLaunchKernelGGL(grid8_kernel, dim3(NF), dim3(64), 0, 0, d);
                else hipLaunchKernelGGL(grid16_kernel, dim3(NF), dim3(64), 0, 0, d);
            }
            (void)hipEventRecord(e1, 0);
            (void)hipEventSynchronize(e1);
            float ms;
            (void)hipEventElapsedTime(&ms, e0, e1);
            med[g][r] = ms * 1e3f / reps;
            if (med[g][r] < best[g]) best[g] = med[g][r];
        }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    for (int g = 0; g < 2; ++g) {
        printf("%s grid: trailing update over pivots 1..52, %d frames:", g == 0 ? "8x8 " : "4x16", NF);
        for (int r = 0; r < rounds; ++r) printf(" %.1f", med[g][r]);
        printf(" us (best %.1f)\n", best[g]);
    }
    return 0;
}
