// wce_ldconv.hip -- the reference's data format on the device.
//
// The reference keeps every array as `long double complex` (main.c:4-8,
// utils.h): on x86-64 that is two x87 80-bit extended values, each in a 16-B
// slot (bytes 0-7 the 64-bit significand with its explicit integer bit,
// bytes 8-9 sign and 15-bit exponent, bytes 10-15 padding that C leaves
// unspecified).  A host that holds frames in that format can copy the raw
// bytes to HBM and convert there, instead of converting value by value on
// the CPU (what the compat shims of wce_compat.cpp do for one frame):
//
//   ldc_to_complex: x87 extended -> fp64, rounded to nearest-even exactly as
//                   the C cast (double)x does on x86 (fld tbyte; fstp qword),
//                   including overflow to Inf, gradual underflow to fp64
//                   subnormals, NaN payload truncation with the quiet bit set,
//                   and the invalid encodings (unnormals, pseudo-Inf/NaN) that
//                   the x87 turns into the default NaN;
//   complex_to_ldc: fp64 -> x87 extended, exact (the C cast (long double)x),
//                   padding bytes written as zero.
//
// HBM-bound integer work: one complex per lane, 32 B <-> 16 B, coalesced.
#include <hip/hip_runtime.h>
#include "wce_internal.h"

namespace wce {

// x87 extended (significand m, sign+exponent se) -> fp64 bit pattern
__device__ __forceinline__ uint64_t x87_to_f64_bits(uint64_t m, uint32_t se)
{
    const uint64_t sign = (uint64_t)((se >> 15) & 1u) << 63;
    const int e = (int)(se & 0x7fffu);
    const uint64_t kIndefinite = 0xfff8000000000000ull;   // the x87 default NaN
    const bool jbit = (m >> 63) != 0;
    if (e == 0x7fff) {
        if (!jbit) return kIndefinite;                               // pseudo-Inf / pseudo-NaN: invalid
        const uint64_t frac = m & 0x7fffffffffffffffull;
        if (frac == 0) return sign | 0x7ff0000000000000ull;          // +-Inf
        return sign | 0x7ff0000000000000ull | (1ull << 51) | ((m >> 11) & 0x000fffffffffffffull);   // quiet, truncated
    }
    if (e == 0) return sign;                                         // |x| < 2^-16382: rounds to +-0
    if (!jbit) return kIndefinite;                                   // unnormal: invalid
    const int E = e - 16383;                                         // x = m 2^(E - 63), m in [2^63, 2^64)
    if (E > 1023) return sign | 0x7ff0000000000000ull;               // overflow
    if (E >= -1022) {                                                // normal fp64
        uint64_t q = m >> 11;                                        // 53 bits, leading 1
        const uint64_t rem = m & 0x7ffull;
        if (rem > 0x400ull || (rem == 0x400ull && (q & 1ull))) ++q;
        int eb = E + 1023;
        if (q >> 53) {                                               // rounding carried out: 2^53
            q >>= 1;
            ++eb;
            if (eb >= 0x7ff) return sign | 0x7ff0000000000000ull;
        }
        return sign | ((uint64_t)eb << 52) | (q & 0x000fffffffffffffull);
    }
    // subnormal fp64: x = q 2^-1074 with q = m 2^(E - 63 + 1074) = m >> s
    const int s = -1011 - E;                                         // >= 12
    if (s > 64) return sign;                                         // below half the smallest subnormal
    const uint64_t q = s == 64 ? 0ull : (m >> s);
    const uint64_t half = 1ull << (s - 1);
    const uint64_t rem = s == 64 ? m : (m & ((1ull << s) - 1ull));
    const uint64_t r = (rem > half || (rem == half && (q & 1ull))) ? q + 1ull : q;
    return sign | r;                                                 // r == 2^52 is the smallest normal
}

// fp64 bit pattern -> x87 extended (exact)
__device__ __forceinline__ void f64_bits_to_x87(uint64_t b, uint64_t &m, uint32_t &se)
{
    const uint32_t sign = (uint32_t)(b >> 63) << 15;
    const int e = (int)((b >> 52) & 0x7ffu);
    const uint64_t f = b & 0x000fffffffffffffull;
    if (e == 0x7ff) {
        se = sign | 0x7fffu;
        m = f == 0 ? (1ull << 63) : ((1ull << 63) | (1ull << 62) | (f << 11));   // Inf; NaN made quiet
        return;
    }
    if (e == 0) {
        if (f == 0) { se = sign; m = 0; return; }
        const int lz = __clzll((long long)f);                       // >= 12
        m = f << lz;
        se = sign | (uint32_t)(-1011 - lz + 16383);
        return;
    }
    m = (1ull << 63) | (f << 11);
    se = sign | (uint32_t)(e - 1023 + 16383);
}

// one complex (two 16-B slots in, 16 B out) per lane
__global__ __launch_bounds__(256) void ldc_to_complex_kernel(const uint64_t *__restrict__ src, double *__restrict__ dst,
                                                            int64_t n)
{
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const ulonglong2 re = reinterpret_cast<const ulonglong2 *>(src)[2 * i];
    const ulonglong2 im = reinterpret_cast<const ulonglong2 *>(src)[2 * i + 1];
    double2 v;
    v.x = __longlong_as_double((long long)x87_to_f64_bits(re.x, (uint32_t)(re.y & 0xffffu)));
    v.y = __longlong_as_double((long long)x87_to_f64_bits(im.x, (uint32_t)(im.y & 0xffffu)));
    reinterpret_cast<double2 *>(dst)[i] = v;
}

__global__ __launch_bounds__(256) void complex_to_ldc_kernel(const double *__restrict__ src, uint64_t *__restrict__ dst,
                                                            int64_t n)
{
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const double2 v = reinterpret_cast<const double2 *>(src)[i];
    uint64_t mr, mi;
    uint32_t ser, sei;
    f64_bits_to_x87((uint64_t)__double_as_longlong(v.x), mr, ser);
    f64_bits_to_x87((uint64_t)__double_as_longlong(v.y), mi, sei);
    const ulonglong2 re = make_ulonglong2(mr, ser), im = make_ulonglong2(mi, sei);
    reinterpret_cast<ulonglong2 *>(dst)[2 * i] = re;
    reinterpret_cast<ulonglong2 *>(dst)[2 * i + 1] = im;
}

int launch_ldc_convert(const void *src, void *dst, int64_t n, bool to_complex, void *stream)
{
    if (n <= 0) return WCE_OK;
    const int64_t blocks = (n + 255) / 256;
    if (blocks > 0x7fffffffll) return WCE_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    if (to_complex)
        hipLaunchKernelGGL(ldc_to_complex_kernel, dim3((unsigned)blocks), dim3(256), 0, s,
                           reinterpret_cast<const uint64_t *>(src), reinterpret_cast<double *>(dst), n);
    else
        hipLaunchKernelGGL(complex_to_ldc_kernel, dim3((unsigned)blocks), dim3(256), 0, s,
                           reinterpret_cast<const double *>(src), reinterpret_cast<uint64_t *>(dst), n);
    return hipGetLastError() == hipSuccess ? WCE_OK : WCE_EHIP;
}

}  // namespace wce
