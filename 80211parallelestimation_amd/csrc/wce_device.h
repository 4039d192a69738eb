// wce_device.h -- complex fp64 and wave64 helpers shared by the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace wce {

// ---------------------------------------------------------------- helpers
__device__ __forceinline__ double2 cadd(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double2 csub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ double2 cscale(double2 a, double s) { return make_double2(a.x * s, a.y * s); }
__device__ __forceinline__ double2 cmul(double2 a, double2 b)
{
    return make_double2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}
__device__ __forceinline__ double2 cconj(double2 a) { return make_double2(a.x, -a.y); }
// 1/d: v_rcp_f64 (2^28 ulp) + 2 Newton steps -> correctly rounded in the
// probe (profiles/r01_ubench_rcp.txt); 5 VALU against 11 for an IEEE divide
__device__ __forceinline__ double rcp_nr(double d)
{
    double r = __builtin_amdgcn_rcp(d);
    double e = fma(-d, r, 1.0);
    r = fma(r, e, r);
    e = fma(-d, r, 1.0);
    return fma(r, e, r);
}
// a / b.  Contraction is off here and the fmas are spelled out, so that every
// kernel that divides -- the LS kernels, the fused epilogue -- rounds alike
// whatever consumes the quotient (a kernel that feeds it straight into
// clerp would otherwise fuse the quotient's product into the subtraction),
// and their outputs stay bit-identical to each other.
__device__ __forceinline__ double2 cdiv(double2 a, double2 b)
{
#pragma clang fp contract(off)
    const double inv = rcp_nr(fma(b.x, b.x, b.y * b.y));
    return make_double2(fma(a.x, b.x, a.y * b.y) * inv, fma(a.y, b.x, -(a.x * b.y)) * inv);
}
// lo + (hi - lo) alpha (main.c:86-99's linear interpolation), one rounding order everywhere
__device__ __forceinline__ double2 clerp(double2 lo, double2 hi, double alpha)
{
#pragma clang fp contract(off)
    return make_double2(fma(hi.x - lo.x, alpha, lo.x), fma(hi.y - lo.y, alpha, lo.y));
}
// acc -= l * conj(c)   (4 DFMA)
__device__ __forceinline__ void cmsub_conj(double2 &acc, double2 l, double2 c)
{
    acc.x = fma(-l.x, c.x, acc.x);
    acc.x = fma(-l.y, c.y, acc.x);
    acc.y = fma(-l.y, c.x, acc.y);
    acc.y = fma(l.x, c.y, acc.y);
}
__device__ __forceinline__ double readlane_f64(double v, int lane)
{
    const long long b = __double_as_longlong(v);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), lane);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), lane);
    return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
__device__ __forceinline__ double2 readlane_c(double2 v, int lane)
{
    return make_double2(readlane_f64(v.x, lane), readlane_f64(v.y, lane));
}
__device__ __forceinline__ double2 shfl_xor_c(double2 v, int m)
{
    return make_double2(__shfl_xor(v.x, m, 64), __shfl_xor(v.y, m, 64));
}
__device__ __forceinline__ double2 shfl_c(double2 v, int src)
{
    return make_double2(__shfl(v.x, src, 64), __shfl(v.y, src, 64));
}
__device__ __forceinline__ double2 ld2(const double *p, int64_t idx)
{
    return reinterpret_cast<const double2 *>(p)[idx];
}
__device__ __forceinline__ void st2(double *p, int64_t idx, double2 v)
{
    reinterpret_cast<double2 *>(p)[idx] = v;
}
typedef double v2d __attribute__((ext_vector_type(2)));
// streaming (non-temporal) 16-B load of inputs read once
__device__ __forceinline__ double2 ld2_nt(const double *p, int64_t idx)
{
    const v2d t = __builtin_nontemporal_load(reinterpret_cast<const v2d *>(p) + idx);
    return make_double2(t[0], t[1]);
}
// streaming (non-temporal) 16-B store of outputs nobody re-reads in this kernel
__device__ __forceinline__ void st2_nt(double *p, int64_t idx, double2 v)
{
    v2d t = {v.x, v.y};
    __builtin_nontemporal_store(t, reinterpret_cast<v2d *>(p) + idx);
}

// Sum over the 8 lanes l ^ {8, 16, 32} (same l & 7) without the LDS pipe:
// xor 8 = DPP row_ror:8 inside each 16-lane row, xor 16 / 32 = gfx950's
// v_permlane16/32_swap (swapping a copy with itself pairs lane l with l ^ 16
// / l ^ 32; the two halves of the result sum to x + x^16 / x + x^32).  Same
// pairs and order as the __shfl_xor butterfly, so results are bit-identical.
__device__ __forceinline__ double dpp_ror8(double v)
{
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0x128, 0xf, 0xf, true);   // every lane has a source:
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0x128, 0xf, 0xf, true);   // no materialised old value
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double sum_xor16(double v)
{
    const auto lo = __builtin_amdgcn_permlane16_swap(__double2loint(v), __double2loint(v), false, false);
    const auto hi = __builtin_amdgcn_permlane16_swap(__double2hiint(v), __double2hiint(v), false, false);
    return __hiloint2double(hi[0], lo[0]) + __hiloint2double(hi[1], lo[1]);
}
__device__ __forceinline__ double sum_xor32(double v)
{
    const auto lo = __builtin_amdgcn_permlane32_swap(__double2loint(v), __double2loint(v), false, false);
    const auto hi = __builtin_amdgcn_permlane32_swap(__double2hiint(v), __double2hiint(v), false, false);
    return __hiloint2double(hi[0], lo[0]) + __hiloint2double(hi[1], lo[1]);
}
__device__ __forceinline__ double2 sum_over_p(double2 w)
{
    w.x += dpp_ror8(w.x);
    w.y += dpp_ror8(w.y);
    return make_double2(sum_xor32(sum_xor16(w.x)), sum_xor32(sum_xor16(w.y)));
}

// wave-local LDS ordering (one wave owns the buffer; no workgroup barrier)
__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

}  // namespace wce
