// wce_front.hip -- gfx950 time-domain front end, the GPU
// version of WiFi_blocks_extraction.m:1-11 and WiFi_RX.m:18-30:
//   80-sample OFDM block -> drop the 16-sample cyclic prefix -> 64-point DFT
//   -> circshift(., 26) -> the 53 useful bins, and for the long training field
//   the same on the mean of its two 64-sample copies plus sigma^2.
//
// HBM-bound (1024 B in, 848 B out per block; ~2.3 kflop).  One wave holds 8
// blocks, 8 lanes per block; each lane owns 8 samples.  The 64-point DFT is
// an 8 x 8 Cooley-Tukey: n = 8 n1 + n2, k = k1 + 8 k2,
//   X[k1 + 8 k2] = sum_n2 W8^(n2 k2) W64^(n2 k1) sum_n1 x[8 n1 + n2] W8^(n1 k1)
// stage 1 on lane n2 (8-point DFT in registers), twiddle, an 8x8 transpose
// through LDS (XOR-swizzled, wave-local), stage 2 on lane k1.  Loads are
// 128-B runs per block per instruction; no MFMA (not GEMM-shaped work).
#include <hip/hip_runtime.h>
#include "wce_internal.h"
#include "wce_device.h"

namespace wce {

// W64^m = exp(-2 pi i m / 64), correctly rounded (mpmath, 40 digits)
__constant__ double2 kW64[64] = {
    {0x1.0000000000000p+0, 0x0.0p+0}, {0x1.fd88da3d12526p-1, -0x1.917a6bc29b42cp-4},
    {0x1.f6297cff75cb0p-1, -0x1.8f8b83c69a60bp-3}, {0x1.e9f4156c62ddap-1, -0x1.294062ed59f06p-2},
    {0x1.d906bcf328d46p-1, -0x1.87de2a6aea963p-2}, {0x1.c38b2f180bdb1p-1, -0x1.e2b5d3806f63bp-2},
    {0x1.a9b66290ea1a3p-1, -0x1.1c73b39ae68c8p-1}, {0x1.8bc806b151741p-1, -0x1.44cf325091dd6p-1},
    {0x1.6a09e667f3bcdp-1, -0x1.6a09e667f3bcdp-1}, {0x1.44cf325091dd6p-1, -0x1.8bc806b151741p-1},
    {0x1.1c73b39ae68c8p-1, -0x1.a9b66290ea1a3p-1}, {0x1.e2b5d3806f63bp-2, -0x1.c38b2f180bdb1p-1},
    {0x1.87de2a6aea963p-2, -0x1.d906bcf328d46p-1}, {0x1.294062ed59f06p-2, -0x1.e9f4156c62ddap-1},
    {0x1.8f8b83c69a60bp-3, -0x1.f6297cff75cb0p-1}, {0x1.917a6bc29b42cp-4, -0x1.fd88da3d12526p-1},
    {0x0.0p+0, -0x1.0000000000000p+0}, {-0x1.917a6bc29b42cp-4, -0x1.fd88da3d12526p-1},
    {-0x1.8f8b83c69a60bp-3, -0x1.f6297cff75cb0p-1}, {-0x1.294062ed59f06p-2, -0x1.e9f4156c62ddap-1},
    {-0x1.87de2a6aea963p-2, -0x1.d906bcf328d46p-1}, {-0x1.e2b5d3806f63bp-2, -0x1.c38b2f180bdb1p-1},
    {-0x1.1c73b39ae68c8p-1, -0x1.a9b66290ea1a3p-1}, {-0x1.44cf325091dd6p-1, -0x1.8bc806b151741p-1},
    {-0x1.6a09e667f3bcdp-1, -0x1.6a09e667f3bcdp-1}, {-0x1.8bc806b151741p-1, -0x1.44cf325091dd6p-1},
    {-0x1.a9b66290ea1a3p-1, -0x1.1c73b39ae68c8p-1}, {-0x1.c38b2f180bdb1p-1, -0x1.e2b5d3806f63bp-2},
    {-0x1.d906bcf328d46p-1, -0x1.87de2a6aea963p-2}, {-0x1.e9f4156c62ddap-1, -0x1.294062ed59f06p-2},
    {-0x1.f6297cff75cb0p-1, -0x1.8f8b83c69a60bp-3}, {-0x1.fd88da3d12526p-1, -0x1.917a6bc29b42cp-4},
    {-0x1.0000000000000p+0, 0x0.0p+0}, {-0x1.fd88da3d12526p-1, 0x1.917a6bc29b42cp-4},
    {-0x1.f6297cff75cb0p-1, 0x1.8f8b83c69a60bp-3}, {-0x1.e9f4156c62ddap-1, 0x1.294062ed59f06p-2},
    {-0x1.d906bcf328d46p-1, 0x1.87de2a6aea963p-2}, {-0x1.c38b2f180bdb1p-1, 0x1.e2b5d3806f63bp-2},
    {-0x1.a9b66290ea1a3p-1, 0x1.1c73b39ae68c8p-1}, {-0x1.8bc806b151741p-1, 0x1.44cf325091dd6p-1},
    {-0x1.6a09e667f3bcdp-1, 0x1.6a09e667f3bcdp-1}, {-0x1.44cf325091dd6p-1, 0x1.8bc806b151741p-1},
    {-0x1.1c73b39ae68c8p-1, 0x1.a9b66290ea1a3p-1}, {-0x1.e2b5d3806f63bp-2, 0x1.c38b2f180bdb1p-1},
    {-0x1.87de2a6aea963p-2, 0x1.d906bcf328d46p-1}, {-0x1.294062ed59f06p-2, 0x1.e9f4156c62ddap-1},
    {-0x1.8f8b83c69a60bp-3, 0x1.f6297cff75cb0p-1}, {-0x1.917a6bc29b42cp-4, 0x1.fd88da3d12526p-1},
    {0x0.0p+0, 0x1.0000000000000p+0}, {0x1.917a6bc29b42cp-4, 0x1.fd88da3d12526p-1},
    {0x1.8f8b83c69a60bp-3, 0x1.f6297cff75cb0p-1}, {0x1.294062ed59f06p-2, 0x1.e9f4156c62ddap-1},
    {0x1.87de2a6aea963p-2, 0x1.d906bcf328d46p-1}, {0x1.e2b5d3806f63bp-2, 0x1.c38b2f180bdb1p-1},
    {0x1.1c73b39ae68c8p-1, 0x1.a9b66290ea1a3p-1}, {0x1.44cf325091dd6p-1, 0x1.8bc806b151741p-1},
    {0x1.6a09e667f3bcdp-1, 0x1.6a09e667f3bcdp-1}, {0x1.8bc806b151741p-1, 0x1.44cf325091dd6p-1},
    {0x1.a9b66290ea1a3p-1, 0x1.1c73b39ae68c8p-1}, {0x1.c38b2f180bdb1p-1, 0x1.e2b5d3806f63bp-2},
    {0x1.d906bcf328d46p-1, 0x1.87de2a6aea963p-2}, {0x1.e9f4156c62ddap-1, 0x1.294062ed59f06p-2},
    {0x1.f6297cff75cb0p-1, 0x1.8f8b83c69a60bp-3}, {0x1.fd88da3d12526p-1, 0x1.917a6bc29b42cp-4}};

// Memory policy per variant, chosen by interleaved A/B on the box
// (tools/ab_front.py, profiles/r01_ab_front.txt): the block kernel stages its
// bins through LDS and stores them as one run per wave, with nontemporal loads
// and stores (5.35 -> 5.98 TB/s); the preamble kernel is fastest with plain
// loads and direct stores (nt: 5.85 -> 5.11 TB/s).
template <bool NT>
__device__ __forceinline__ double2 fe_ld(const double2 *p)
{
    if constexpr (NT) {
        const v2d t = __builtin_nontemporal_load(reinterpret_cast<const v2d *>(p));
        return make_double2(t.x, t.y);
    } else {
        return *p;
    }
}
template <bool NT>
__device__ __forceinline__ void fe_st(double2 *p, double2 v)
{
    if constexpr (NT) {
        v2d t = {v.x, v.y};
        __builtin_nontemporal_store(t, reinterpret_cast<v2d *>(p));
    } else {
        *p = v;
    }
}

constexpr int FE_WAVES = 4;      // waves per 256-thread workgroup
constexpr int FE_UNITS = 8;      // blocks per wave iteration

// in-register 8-point DFT, radix-2 (W8^1 = c(1 - i), W8^2 = -i, W8^3 = -c(1 + i))
__device__ __forceinline__ void dft8(double2 (&x)[8])
{
    const double c = 0x1.6a09e667f3bcdp-1;   // sqrt(2)/2
    const double2 b0 = cadd(x[0], x[4]), b1 = csub(x[0], x[4]), b2 = cadd(x[2], x[6]), b3 = csub(x[2], x[6]);
    const double2 b4 = cadd(x[1], x[5]), b5 = csub(x[1], x[5]), b6 = cadd(x[3], x[7]), b7 = csub(x[3], x[7]);
    const double2 e0 = cadd(b0, b2), e2 = csub(b0, b2);
    const double2 e1 = make_double2(b1.x + b3.y, b1.y - b3.x), e3 = make_double2(b1.x - b3.y, b1.y + b3.x);
    const double2 o0 = cadd(b4, b6), o2 = csub(b4, b6);
    const double2 o1 = make_double2(b5.x + b7.y, b5.y - b7.x), o3 = make_double2(b5.x - b7.y, b5.y + b7.x);
    const double2 t1 = make_double2(c * (o1.x + o1.y), c * (o1.y - o1.x));
    const double2 t2 = make_double2(o2.y, -o2.x);
    const double2 t3 = make_double2(c * (o3.y - o3.x), -c * (o3.x + o3.y));
    x[0] = cadd(e0, o0); x[4] = csub(e0, o0);
    x[1] = cadd(e1, t1); x[5] = csub(e1, t1);
    x[2] = cadd(e2, t2); x[6] = csub(e2, t2);
    x[3] = cadd(e3, t3); x[7] = csub(e3, t3);
}

// PRE = false: unit = OFDM block (80 samples, CP 16).  PRE = true: unit =
// one frame's long training field (two 64-sample copies at a.off, a.off + 64).
template <bool PRE>
__global__ __launch_bounds__(256) void front_kernel(FrontArgs a)
{
    __shared__ double2 lds[FE_WAVES][FE_UNITS][64];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int g = lane >> 3, j = lane & 7;
    double2 *T = lds[w][g];
    const double2 *src = reinterpret_cast<const double2 *>(a.src);
    double2 *dst = reinterpret_cast<double2 *>(a.dst);
    constexpr bool NT = !PRE, STAGED = !PRE;
    double2 tw[8];
#pragma unroll
    for (int k1 = 0; k1 < 8; ++k1) tw[k1] = kW64[(j * k1) & 63];
    const uint32_t stride = gridDim.x * FE_WAVES * FE_UNITS;
    for (uint32_t u0 = (blockIdx.x * FE_WAVES + w) * FE_UNITS; u0 < a.n_units; u0 += stride) {
        const bool live = u0 + g < a.n_units;
        const uint32_t u = live ? u0 + g : a.n_units - 1;
        const uint32_t f = u / a.nb, b = u - f * a.nb;
        const double2 *x = src + (int64_t)f * a.ps + a.off + (int64_t)b * 80 + j;
        double2 v[8];
        double s2 = 0.0;
        if constexpr (PRE) {      // WiFi_RX.m:24-30: p2 = x[0..64), p1 = x[64..128)
            double2 p2[8], p1[8];
#pragma unroll
            for (int n1 = 0; n1 < 8; ++n1) { p2[n1] = fe_ld<NT>(x + 8 * n1); p1[n1] = fe_ld<NT>(x + 64 + 8 * n1); }
#pragma unroll
            for (int n1 = 0; n1 < 8; ++n1) {
                v[n1] = cscale(cadd(p1[n1], p2[n1]), 0.5);
                const double2 d = csub(p2[n1], p1[n1]);
                s2 += d.x * d.x + d.y * d.y;
            }
        } else {
#pragma unroll
            for (int n1 = 0; n1 < 8; ++n1) v[n1] = fe_ld<NT>(x + 8 * n1);
        }
        // stage 1 (lane = n2): DFT over n1, then W64^(n2 k1)
        dft8(v);
#pragma unroll
        for (int k1 = 1; k1 < 8; ++k1) v[k1] = cmul(v[k1], tw[k1]);
        // transpose: element (n2, k1) at n2 * 8 + (k1 ^ n2)
#pragma unroll
        for (int k1 = 0; k1 < 8; ++k1) T[j * 8 + (k1 ^ j)] = v[k1];
        wave_lds_sync();
#pragma unroll
        for (int n2 = 0; n2 < 8; ++n2) v[n2] = T[n2 * 8 + (j ^ n2)];
        wave_lds_sync();
        // stage 2 (lane = k1): DFT over n2 -> bin k = k1 + 8 k2
        dft8(v);
        if constexpr (STAGED) {
            // stage the 8 x 53 bins in LDS, then store them as one run per wave
            // (contiguous when consecutive blocks are adjacent, block_stride 53)
#pragma unroll
            for (int k2 = 0; k2 < 8; ++k2) T[(j + 8 * k2 + 26) & 63] = v[k2];
            wave_lds_sync();
#pragma unroll
            for (int t = 0; t < (FE_UNITS * NSC + 63) / 64; ++t) {
                const int e = lane + 64 * t;
                const int ug = e / NSC, i = e - ug * NSC;
                const uint32_t uu = u0 + ug;
                if (e < FE_UNITS * NSC && uu < a.n_units) {
                    const uint32_t ff = uu / a.nb, bb = uu - ff * a.nb;
                    fe_st<NT>(dst + (int64_t)ff * a.fs + (int64_t)bb * a.bs + i, lds[w][ug][i]);
                }
            }
            wave_lds_sync();
        } else {
            double2 *y = dst + (int64_t)f * a.fs + (int64_t)b * a.bs;
#pragma unroll
            for (int k2 = 0; k2 < 8; ++k2) {
                const int i = (j + 8 * k2 + 26) & 63;   // circshift(., 26), keep 1:53
                if (live && i < NSC) fe_st<NT>(y + i, v[k2]);
            }
        }
        if constexpr (PRE) {
            if (a.ow2) {
                s2 += __shfl_xor(s2, 1, 64);
                s2 += __shfl_xor(s2, 2, 64);
                s2 += __shfl_xor(s2, 4, 64);
                if (live && j == 0) a.ow2[f] = s2 / 128.0;   // 2 K, K = 64
            }
        }
    }
}

int launch_front(const FrontArgs &a, bool preamble, void *stream)
{
    if (a.n_units == 0) return 0;
    const uint32_t units_per_wg = FE_WAVES * FE_UNITS;
    uint32_t blocks = (a.n_units + units_per_wg - 1) / units_per_wg;
    if (blocks > 256u * 40u) blocks = 256u * 40u;   // grid-stride beyond ~40 workgroups per CU
    const dim3 grid(blocks), blk(256);
    if (preamble)
        hipLaunchKernelGGL(front_kernel<true>, grid, blk, 0, (hipStream_t)stream, a);
    else
        hipLaunchKernelGGL(front_kernel<false>, grid, blk, 0, (hipStream_t)stream, a);
    return hipGetLastError() == hipSuccess ? WCE_OK : WCE_EHIP;
}

}  // namespace wce
