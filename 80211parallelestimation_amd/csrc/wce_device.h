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


// a = c on the lanes of mask m (a constant) that are active: two v_mov_b64 under EXEC
__device__ __forceinline__ void keep_where_mask(uint64_t m, bool sel, double2 &a, double2 c)
{
    uint64_t sv;
    asm volatile("s_mov_b64 %[sv], exec\n\t"
                 "s_mov_b64 exec, %[m]\n\t"
                 "v_mov_b64 %[ax], %[cx]\n\t"
                 "v_mov_b64 %[ay], %[cy]\n\t"
                 "s_mov_b64 exec, %[sv]"
                 : [ax] "+v"(a.x), [ay] "+v"(a.y), [sv] "=&s"(sv)
                 : [m] "s"(m & __builtin_amdgcn_read_exec()), [cx] "v"(c.x), [cy] "v"(c.y));
}
// lanes with (lane & 15) <= c / == c in every 16-lane row
constexpr uint64_t rows16_upto(int c) { return ((2ull << c) - 1) * 0x0001000100010001ull; }
constexpr uint64_t rows16_at(int c) { return 0x0001000100010001ull << c; }

// ---------------------------------------------------------------- shared by the kernel files
// 1/sqrt(d) from v_rsq_f64 (relative error ~2^-24).  One third-order
// (Householder) step y += y e (1/2 + 3e/8), e = 1 - d y^2: error ~2^-72
// before rounding, 5 VALU on a 4-deep chain (two Newton steps: 7 on 6, 2.1%
// slower, retired in round 4).
__device__ __forceinline__ double rsq_nr(double d)
{
    const double y = __builtin_amdgcn_rsq(d);
    const double e = fma(-d * y, y, 1.0);
    return fma(y * e, fma(e, 0.375, 0.5), y);
}

// 53-point DFTs on lane m: E[k m mod 53] gathered by byte offset, the step m * 16
// added, 848 subtracted when it
// wraps -- min_u32(o + s, o + s - 848) (the wrapped value underflows to a huge
// unsigned when no wrap is due): three integer ops and no shift per gather
__device__ __forceinline__ uint32_t dft_step(uint32_t o, uint32_t s, uint32_t s_wrap)
{
    return min(o + s, o + s_wrap);
}
__device__ __forceinline__ double2 ld_e(const double2 *e, uint32_t o)
{
    return *reinterpret_cast<const double2 *>(reinterpret_cast<const char *>(e) + o);
}

template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v)
{
    // every lane of the 16-lane row reads a valid source lane for the controls
    // used here (row_newbcast, quad_perm, mirrors), so no "old" value is needed:
    // mov_dpp is one v_mov_b32_dpp per half, where update_dpp(0, ...) also
    // materialised the zero (a v_mov_b32 per half)
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xf, 0xf, true);
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xf, 0xf, true);
    return __hiloint2double(hi, lo);
}
template <int N>
__device__ __forceinline__ double2 row_bcast(double2 v)   // lane N of each 16-lane row, to the row
{
    return make_double2(dpp_f64<0x150 + N>(v.x), dpp_f64<0x150 + N>(v.y));
}
__device__ __forceinline__ double row16_sum(double v)   // over a 16-lane row, the same bits in every lane
{
    v += dpp_f64<0xB1>(v);    // quad_perm [1,0,3,2]
    v += dpp_f64<0x4E>(v);    // quad_perm [2,3,0,1]
    v += dpp_f64<0x141>(v);   // row_half_mirror
    v += dpp_f64<0x140>(v);   // row_mirror
    return v;
}
__device__ __forceinline__ double2 row16_sum(double2 v) { return make_double2(row16_sum(v.x), row16_sum(v.y)); }

__device__ __forceinline__ double2 row_bcast_n(double2 v, int n)   // n a constant after unrolling
{
    switch (n) {
    case 0: return row_bcast<0>(v);
    case 1: return row_bcast<1>(v);
    case 2: return row_bcast<2>(v);
    case 3: return row_bcast<3>(v);
    case 4: return row_bcast<4>(v);
    case 5: return row_bcast<5>(v);
    case 6: return row_bcast<6>(v);
    case 7: return row_bcast<7>(v);
    case 8: return row_bcast<8>(v);
    case 9: return row_bcast<9>(v);
    case 10: return row_bcast<10>(v);
    case 11: return row_bcast<11>(v);
    case 12: return row_bcast<12>(v);
    case 13: return row_bcast<13>(v);
    case 14: return row_bcast<14>(v);
    default: return row_bcast<15>(v);
    }
}

// ---------------------------------------------------------------- DPP64 FMAs (quad kernels)
// acc -= l conj(R[lane N of the 16-lane row]): gfx950's DPP64 row_newbcast on
// v_fmac_f64 hands the broadcast operand straight to the FMA (4 VALU instead
// of 2 v_mov_b64_dpp + 4 FMAs), the products and their order those of
// cmsub_conj.  R must not have been written by a VALU instruction in the 2
// wait states before (dpp_ready below).
template <int N>
__device__ __forceinline__ void cmsub_dpp(double2 &acc, double2 l, double2 R)
{
    asm("v_fmac_f64_dpp %[ax], -%[cx], %[lx] row_newbcast:%c[n] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %[ax], -%[cy], %[ly] row_newbcast:%c[n] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %[ay], -%[cx], %[ly] row_newbcast:%c[n] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %[ay], %[cy], %[lx] row_newbcast:%c[n] row_mask:0xf bank_mask:0xf"
        : [ax] "+v"(acc.x), [ay] "+v"(acc.y)
        : [lx] "v"(l.x), [ly] "v"(l.y), [cx] "v"(R.x), [cy] "v"(R.y), [n] "i"(N));
}
__device__ __forceinline__ void cmsub_dpp_n(int n, double2 &acc, double2 l, double2 R)   // n constant after unrolling
{
    switch (n) {
    case 0: cmsub_dpp<0>(acc, l, R); break;
    case 1: cmsub_dpp<1>(acc, l, R); break;
    case 2: cmsub_dpp<2>(acc, l, R); break;
    case 3: cmsub_dpp<3>(acc, l, R); break;
    case 4: cmsub_dpp<4>(acc, l, R); break;
    case 5: cmsub_dpp<5>(acc, l, R); break;
    case 6: cmsub_dpp<6>(acc, l, R); break;
    case 7: cmsub_dpp<7>(acc, l, R); break;
    case 8: cmsub_dpp<8>(acc, l, R); break;
    case 9: cmsub_dpp<9>(acc, l, R); break;
    case 10: cmsub_dpp<10>(acc, l, R); break;
    case 11: cmsub_dpp<11>(acc, l, R); break;
    case 12: cmsub_dpp<12>(acc, l, R); break;
    case 13: cmsub_dpp<13>(acc, l, R); break;
    case 14: cmsub_dpp<14>(acc, l, R); break;
    default: cmsub_dpp<15>(acc, l, R); break;
    }
}
// the 2 wait states between the VALU write of a DPP source and its first DPP
// read, tied to the values so nothing moves across it
__device__ __forceinline__ void dpp_ready(double2 &a, double2 &b)
{
    asm volatile("s_nop 1" : "+v"(a.x), "+v"(a.y), "+v"(b.x), "+v"(b.y));
}
__device__ __forceinline__ void dpp_ready(double2 &a)
{
    asm volatile("s_nop 1" : "+v"(a.x), "+v"(a.y));
}
// A += c[lane N] Re e, B += c[lane N] Im e (the read-out pairs), c as the DPP64
// row_newbcast operand of the four FMAs; c ready as for cmsub_dpp
template <int N>
__device__ __forceinline__ void cfma_dpp(double2 &A, double2 &B, double2 c, double2 e)
{
    asm("v_fmac_f64_dpp %[ax], %[cx], %[er] row_newbcast:%c[n] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %[ay], %[cy], %[er] row_newbcast:%c[n] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %[bx], %[cx], %[ei] row_newbcast:%c[n] row_mask:0xf bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %[by], %[cy], %[ei] row_newbcast:%c[n] row_mask:0xf bank_mask:0xf"
        : [ax] "+v"(A.x), [ay] "+v"(A.y), [bx] "+v"(B.x), [by] "+v"(B.y)
        : [cx] "v"(c.x), [cy] "v"(c.y), [er] "v"(e.x), [ei] "v"(e.y), [n] "i"(N));
}
__device__ __forceinline__ void cfma_dpp_n(int n, double2 &A, double2 &B, double2 c, double2 e)
{
    switch (n) {
    case 0: cfma_dpp<0>(A, B, c, e); break;
    case 1: cfma_dpp<1>(A, B, c, e); break;
    case 2: cfma_dpp<2>(A, B, c, e); break;
    case 3: cfma_dpp<3>(A, B, c, e); break;
    case 4: cfma_dpp<4>(A, B, c, e); break;
    case 5: cfma_dpp<5>(A, B, c, e); break;
    case 6: cfma_dpp<6>(A, B, c, e); break;
    case 7: cfma_dpp<7>(A, B, c, e); break;
    case 8: cfma_dpp<8>(A, B, c, e); break;
    case 9: cfma_dpp<9>(A, B, c, e); break;
    case 10: cfma_dpp<10>(A, B, c, e); break;
    case 11: cfma_dpp<11>(A, B, c, e); break;
    case 12: cfma_dpp<12>(A, B, c, e); break;
    case 13: cfma_dpp<13>(A, B, c, e); break;
    case 14: cfma_dpp<14>(A, B, c, e); break;
    default: cfma_dpp<15>(A, B, c, e); break;
    }
}
// the read-out's column j (compile-time, so each DPP lane select is an
// immediate): c_j from lane j of ca (j < 16) or lane j - 16 of cb
template <int R, int J>
__device__ __forceinline__ void lrq2_readout(const double2 *sE, double2 ca, double2 cb, uint32_t &o1, uint32_t &o2,
                                             uint32_t s1, uint32_t w1, uint32_t s2, uint32_t w2, double2 &A1,
                                             double2 &B1, double2 &A2, double2 &B2)
{
    if constexpr (J < R) {
        const double2 e1 = ld_e(sE, o1), e2 = ld_e(sE, o2);
        if constexpr (J < 16) {
            cfma_dpp<J>(A1, B1, ca, e1);
            cfma_dpp<J>(A2, B2, ca, e2);
        } else {
            cfma_dpp<J - 16>(A1, B1, cb, e1);
            cfma_dpp<J - 16>(A2, B2, cb, e2);
        }
        o1 = dft_step(o1, s1, w1);
        o2 = dft_step(o2, s2, w2);
        lrq2_readout<R, J + 1>(sE, ca, cb, o1, o2, s1, w1, s2, w2, A1, B1, A2, B2);
    }
}

// Complex symbols in the quad kernels' tap domain (U[k][j] = s_j E[k j]; round 6):
//   s = t + U^H [(x - conj x) o (rx - a x o (U t))] / b
// with U t the read-out DFT of c = s o t (the lane's subcarriers k1 = i + 1,
// 53 - k1 and, for i <= 9, k2 = i + 17, 53 - k2; k = 0 on lane 0) and U^H v
// the Gram's beta DFT of v over the (k, 53 - k) pairs: three DFTs where the
// row form spent R broadcasts, 4R products and R 16-lane sums on each side.
// xm: State::xmask; tx / rx: the unit's block at base.  In: ca / cb = c on rows i and i + 16 (two
// variables; cb a copy of ca when R <= 16).  Out: ca / cb =
// (U^H v)_i / b and (U^H v)_{i+16} / b without the s factor (the caller adds
// s_i times it to t_i).  V: 53 dead entries of the unit's LDS (v, then its pair
// tables in place).
template <int R>
__device__ __forceinline__ void lrq_cplx_taps(uint64_t xm, const double *tx, const double *rx, int64_t base,
                                              const double2 *sE, double2 *V, double2 &ca, double2 &cb, int i,
                                              double ac, double bc)
{
    constexpr int NSC = 53;
    const int k1 = i + 1, k2 = i + 17;
    const bool two = k2 <= NSC / 2;
    double2 h0;
    if constexpr (R > 16) h0 = row16_sum(cadd(ca, cb));
    else h0 = row16_sum(ca);
    {   // y = U t at the lane's subcarriers
        const uint32_t s1 = 16u * (uint32_t)k1, w1 = s1 - 16u * NSC;
        const uint32_t s2 = 16u * (uint32_t)(two ? k2 : k1), w2 = s2 - 16u * NSC;
        uint32_t o1 = 0, o2 = 0;
        double2 A1 = make_double2(0.0, 0.0), B1 = A1, A2 = A1, B2 = A1;
        dpp_ready(ca, cb);
        lrq2_readout<R, 0>(sE, ca, cb, o1, o2, s1, w1, s2, w2, A1, B1, A2, B2);
        const int ks[5] = {k1, NSC - k1, two ? k2 : k1, two ? NSC - k2 : NSC - k1, 0};
        const double2 ys[5] = {make_double2(A1.x - B1.y, A1.y + B1.x), make_double2(A1.x + B1.y, A1.y - B1.x),
                               make_double2(A2.x - B2.y, A2.y + B2.x), make_double2(A2.x + B2.y, A2.y - B2.x), h0};
        double2 xs[5], rs[5];
#pragma unroll
        for (int m = 0; m < 5; ++m) {   // all loads first: one memory round trip
            xs[m] = ld2(tx, base + ks[m]);
            rs[m] = ld2(rx, base + ks[m]);
        }
#pragma unroll
        for (int m = 0; m < 5; ++m) {   // v_k = (x - conj x) (rx - a x y_k) = 2 i Im(x) rho
            if ((m == 2 || m == 3) && !two) continue;
            if (m == 4 && i != 0) continue;
            const double2 x = ((xm >> ks[m]) & 1ull) ? xs[m] : make_double2(0.0, 0.0);
            const double2 rho = csub(rs[m], cscale(cmul(x, ys[m]), ac));
            V[ks[m]] = make_double2(-2.0 * x.y * rho.y, 2.0 * x.y * rho.x);
        }
    }
    wave_lds_sync();
    {   // pair tables of v in place, k = 1..26: V[k] = v_k + v_{53-k}, V[53-k] = v_k - v_{53-k}
        double2 u[2], w[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int kp = i + 1 + 16 * h, kc = kp <= NSC / 2 ? kp : 1;
            u[h] = V[kc];
            w[h] = V[NSC - kc];
        }
        wave_lds_sync();
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int kp = i + 1 + 16 * h;
            if (kp <= NSC / 2) {
                V[kp] = cadd(u[h], w[h]);
                V[NSC - kp] = csub(u[h], w[h]);
            }
        }
    }
    wave_lds_sync();
    // (U^H v)_r / s_r = sum_k v_k conj(E[k r]) at r = i and i + 16
    double2 ba = V[0], bb = ba;
    const uint32_t sa = 16u * (uint32_t)i, swa = sa - 16u * NSC;
    const uint32_t sb = 16u * (uint32_t)(i + 16), swb = sb - 16u * NSC;
    uint32_t oa = sa, ob = sb;
#pragma unroll 2
    for (int k = 1; k <= NSC / 2; ++k) {
        const double2 ea = ld_e(sE, oa), pa = V[k], pb = V[NSC - k];
        ba.x = fma(pa.x, ea.x, fma(pb.y, ea.y, ba.x));
        ba.y = fma(pa.y, ea.x, fma(-pb.x, ea.y, ba.y));
        if constexpr (R > 16) {
            const double2 eb = ld_e(sE, ob);
            bb.x = fma(pa.x, eb.x, fma(pb.y, eb.y, bb.x));
            bb.y = fma(pa.y, eb.x, fma(-pb.x, eb.y, bb.y));
            ob = dft_step(ob, sb, swb);
        }
        oa = dft_step(oa, sa, swa);
    }
    const double rb = 1.0 / bc;
    ca = cscale(ba, rb);
    cb = cscale(bb, rb);
}

}  // namespace wce
