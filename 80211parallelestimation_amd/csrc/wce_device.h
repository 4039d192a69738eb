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
__device__ __forceinline__ double2 cdiv(double2 a, double2 b)
{
    const double inv = 1.0 / (b.x * b.x + b.y * b.y);
    return make_double2((a.x * b.x + a.y * b.y) * inv, (a.y * b.x - a.x * b.y) * inv);
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
// streaming (non-temporal) 16-B store of outputs nobody re-reads in this kernel
__device__ __forceinline__ void st2_nt(double *p, int64_t idx, double2 v)
{
    v2d t = {v.x, v.y};
    __builtin_nontemporal_store(t, reinterpret_cast<v2d *>(p) + idx);
}

// wave-local LDS ordering (one wave owns the buffer; no workgroup barrier)
__device__ __forceinline__ void wave_lds_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

}  // namespace wce
