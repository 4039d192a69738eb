// wce_kernels.hip -- gfx950 (CDNA4) kernels of the 802.11 channel-estimation
// engine.  Written for wave64 / MI355X only.
//
//   ls_kernel             LT_LS + PS_Linear/Cubic/Sinc + equalization, one
//                         wave per frame, HBM streaming (main.c:66-146,
//                         WiFi_Equalization.m); C or MATLAB semantics.
//   ls_elem_kernel        LT_LS + PS_Linear only (BASELINE configs[1]), C
//                         semantics, one (frame, subcarrier) element per thread.
//   mmse_ref_flat_kernel  PS_MMSE in main.c semantics (diagonal Ryy: 4 pilot
//                         terms per frame, H = u s), flat elements, HBM-bound.
//   solve_block           the per-frame MMSE core: Ryy = a X C X' + b I built
//                         in registers (8x8 lane grid, block-cyclic 28 blocks)
//                         with conj(rx) bordered on as row 53 (forward solve
//                         for free), LDS for the pivot-column broadcast
//                         (main.c:148-212 / WiFi_channel_estimation_PS_MMSE.m).
//                         Two read-outs:
//   mmse_solve_fc_kernel    rank-1 C = u w^T (TEXTBOOK, per-frame C; the
//                           headline): Cholesky with row-per-lane panels (one
//                           full-wave publish per pivot, dot_factor); a second
//                           bordered row (w o x)^T leaves s = w^T X z in the
//                           Schur complement; H = u s, one launch.
//   mmse_solve_kernel       dense C (COV): row-per-lane Cholesky keeping L,
//                           blocked back-substitution, W = X z;
//   apply_kernel            then H = C W on v_mfma_f64_16x16x4_f64 + 4x4x4_4b
//                           (persistent, C staged in LDS, 3M complex form).
//   matvec_kernel         the same MFMA product with M from L2: the per-frame
//                         covariance factor u = Mu h, MATLAB's block mean.
//   ref_fc_kernel         REF PS_MMSE with each frame's own LT_LS covariance
//                         (main.c:37-53 + 148-212), one persistent launch.
//   cm_real_kernel        constant-modulus operator H = K (conj(x) o rx).
//   mmse_solve_ls_kernel  config 5: either solve with the LS family and
//                         equalization of the same frame in its epilogue.
//   fc_finish_kernel      MATLAB averaging of the per-block s values.
//   synth_kernel          counter-RNG synthetic frames (bench / tests).
// The time-domain front end is in wce_front.hip.
#include <hip/hip_runtime.h>
#include "wce_internal.h"
#include "wce_device.h"

namespace wce {

// =====================================================================
// LS family + equalization: one wave per frame, lane k = subcarrier k.
// =====================================================================
constexpr int LS_WAVES = 4;   // waves per 256-thread workgroup
constexpr int LS_FRAMES = 4;  // frames per wave iteration: all loads issued up front

// Per-lane (subcarrier k) constants of the LS family, shared by ls_kernel and
// the fused MMSE epilogue.
struct LsLane {
    double2 tpk, tden, hlt_shared;
    double cq, s0, s1, s2, s3, alpha, dk0, dk1, dk2;
    int seg;
};
__device__ __forceinline__ LsLane ls_lane(const State *__restrict__ st, const double *tx_pre, int k)
{
    LsLane c;
    const double *txp = tx_pre ? tx_pre : st->tx_pre;
    c.tpk = ld2(txp, k);
    c.cq = c.tpk.x - c.tpk.y;                  // real "conj" of main.c:69-70
    c.tden = make_double2(c.cq * c.tpk.x, c.cq * c.tpk.y);
    c.hlt_shared = ld2(st->h_lt, k);
    c.s0 = st->sinc[0][k]; c.s1 = st->sinc[1][k]; c.s2 = st->sinc[2][k]; c.s3 = st->sinc[3][k];
    // linear interpolation segment (main.c:86-99): k < 19 seg 0, k < 33 seg 1, else seg 2
    c.seg = k < WCE_P1 ? 0 : (k < WCE_P2 ? 1 : 2);
    c.alpha = (double)(k - (c.seg == 0 ? WCE_P0 : (c.seg == 1 ? WCE_P1 : WCE_P2))) * (1.0 / 14.0);
    c.dk0 = (double)(k - WCE_P0); c.dk1 = (double)(k - WCE_P1); c.dk2 = (double)(k - WCE_P2);
    return c;
}

// LT_LS of subcarrier k from the frame's preamble rp (or the shared one)
template <bool ML>
__device__ __forceinline__ double2 lt_ls_lane(const LsLane &c, bool have_rp, double2 rp, int k)
{
    double2 hlt = c.hlt_shared;
    if (have_rp) {
        if (ML)   // WiFi_channel_estimation_LT_LS.m: conj(tx) rx / (conj(tx) tx)
            hlt = cscale(cmul(cconj(c.tpk), rp), 1.0 / (c.tpk.x * c.tpk.x + c.tpk.y * c.tpk.y));
        else      // main.c:69-72: real "conj" c = re - im
            hlt = cdiv(make_double2(c.cq * rp.x, c.cq * rp.y), c.tden);
    }
    return k == WCE_DC ? make_double2(0, 0) : hlt;   // main.c:74
}

// PS_Linear / PS_Cubic / PS_Sinc of subcarrier k from the pilot LS h0..h3
template <bool ML>
__device__ __forceinline__ void ps_lane(const LsLane &c, uint32_t mask, double2 h0, double2 h1, double2 h2,
                                        double2 h3, double2 &hlin, double2 &hcub, double2 &hsnc)
{
    hlin = hcub = hsnc = make_double2(0, 0);
    if (mask & (WCE_EST_PS_LINEAR | WCE_EQUALIZE)) {      // main.c:86-99
        const double2 lo = c.seg == 0 ? h0 : (c.seg == 1 ? h1 : h2);
        const double2 hi = c.seg == 0 ? h1 : (c.seg == 1 ? h2 : h3);
        hlin = clerp(lo, hi, c.alpha);
    }
    if (mask & WCE_EST_PS_CUBIC) {         // main.c:112-121, every divisor 14
        const double r = 1.0 / 14.0;     // MATLAB (PS_Cubic.m:11-13): 14, 28, 42
        const double r2 = ML ? 1.0 / 28.0 : r, r3 = ML ? 1.0 / 42.0 : r;
        const double2 f01 = cscale(csub(h1, h0), r), f12 = cscale(csub(h2, h1), r), f23 = cscale(csub(h3, h2), r);
        const double2 f012 = cscale(csub(f12, f01), r2), f123 = cscale(csub(f23, f12), r2);
        const double2 f0123 = cscale(csub(f123, f012), r3);
        hcub = cadd(cadd(cadd(h0, cscale(f01, c.dk0)), cscale(cscale(f012, c.dk0), c.dk1)),
                    cscale(cscale(cscale(f0123, c.dk0), c.dk1), c.dk2));
    }
    if (mask & WCE_EST_PS_SINC)            // main.c:135-145
        hsnc = cadd(cadd(cadd(cscale(h0, c.s0), cscale(h1, c.s1)), cscale(h2, c.s2)), cscale(h3, c.s3));
}

// store the requested LS-family outputs of frame f, subcarrier k, and run
// WiFi_Equalization.m:1-9 over the frame's 15 blocks
typedef float v2f __attribute__((ext_vector_type(2)));
// one output element: complex double, or complex float (WCE_OUT_LS_F32)
__device__ __forceinline__ void st_out(double *p, int64_t idx, double2 v, bool f32)
{
    if (f32) {
        v2f t = {(float)v.x, (float)v.y};
        __builtin_nontemporal_store(t, reinterpret_cast<v2f *>(p) + idx);
    } else {
        st2_nt(p, idx, v);
    }
}

// store the requested LS-family outputs of frame f, subcarrier k, and run
// WiFi_Equalization.m:1-9 over the frame's 15 blocks rv (already loaded)
template <bool EQ>
__device__ __forceinline__ void ls_store_rv(const LsArgs &a, int64_t f, int k, uint32_t mask, double2 hlt, double2 hlin,
                                            double2 hcub, double2 hsnc, const double2 (&rv)[NBLK])
{
    const int64_t o = f * a.os + k;
    const bool f32 = a.f32 != 0;
    if ((mask & WCE_EST_LT_LS) && a.lt) st_out(a.lt, o, hlt, f32);
    if ((mask & WCE_EST_PS_LINEAR) && a.lin) st_out(a.lin, o, hlin, f32);
    if ((mask & WCE_EST_PS_CUBIC) && a.cub) st_out(a.cub, o, hcub, f32);
    if ((mask & WCE_EST_PS_SINC) && a.snc) st_out(a.snc, o, hsnc, f32);
    if constexpr (EQ) {
        const double2 hps = a.eq_src == WCE_EST_PS_CUBIC ? hcub : (a.eq_src == WCE_EST_PS_SINC ? hsnc : hlin);
        const int64_t eb = f * a.eqfs + k;
        if (f32) {   // fp32 outputs: the equalizer's divisions in fp32
            // WCE_OUT_LS_F32 (BASELINE configs[4]'s fp32 interpolation stage): the
            // 15 divisions in fp32.  H_UTIL_b = hlt + ((b+1)/15)(hps - hlt) stays
            // fp64 (one fma per component: the blend cancels where the channel
            // fades -- fp32 there is 7e-6 off), scaled by 2^-e, e the exponent of
            // the larger of |hlt|, |hps| (exact, and |H_UTIL|^2 stays inside fp32's
            // range), then rounded to fp32; rx_b is rounded to fp32 and scaled
            // alike; rx / H_UTIL by v_rcp_f32 (1 ulp).  A numpy model of these
            // roundings: <= 4.0e-7 norm-relative from the fp64 quotient over 40,000
            // frames (G4 allows 1e-6; tests/test_config5_gpu.py checks it).
            // WiFi_Equalization.m:3-8.
            const double2 dps = csub(hps, hlt);
            int e = 0;
            (void)frexp(fmax(fmax(fabs(hlt.x), fabs(hlt.y)), fmax(fabs(hps.x), fabs(hps.y))), &e);
            e = e < -120 ? -120 : (e > 120 ? 120 : e);
            const double sc = ldexp(1.0, -e);
            const float sf = (float)sc;
            const double2 h0s = cscale(hlt, sc), d0s = cscale(dps, sc);
#pragma unroll
            for (int b = 0; b < NBLK; b++) {
                const double t = (double)(b + 1) / NBLK;
                const float ur = (float)fma(d0s.x, t, h0s.x), ui = (float)fma(d0s.y, t, h0s.y);
                const float xr = (float)rv[b].x * sf, xi = (float)rv[b].y * sf;
                const float inv = __builtin_amdgcn_rcpf(fmaf(ur, ur, ui * ui));
                v2f q = {fmaf(xr, ur, xi * ui) * inv, fmaf(xi, ur, -(xr * ui)) * inv};
                if (k == WCE_DC) q = v2f{0.0f, 0.0f};
                __builtin_nontemporal_store(q, reinterpret_cast<v2f *>(a.eq) + eb + b * a.eqbs);
            }
            return;
        }
#pragma unroll
        for (int b = 0; b < NBLK; b++) {
            const double wlt = (double)(NBLK - (b + 1)) / NBLK, wps = (double)(b + 1) / NBLK;
            const double2 hu = cadd(cscale(hlt, wlt), cscale(hps, wps));
            const double2 e = k == WCE_DC ? make_double2(0, 0) : cdiv(rv[b], hu);
            st_out(a.eq, eb + b * a.eqbs, e, f32);
        }
    }
}
template <bool EQ>
__device__ __forceinline__ void ls_store(const LsArgs &a, int64_t f, int k, uint32_t mask, double2 hlt, double2 hlin,
                                         double2 hcub, double2 hsnc)
{
    double2 rv[NBLK];
    if constexpr (EQ) {
#pragma unroll
        for (int b = 0; b < NBLK; b++)
            rv[b] = ld2_nt(a.rx, f * a.fs + k + b * a.bs);
    }
    ls_store_rv<EQ>(a, f, k, mask, hlt, hlin, hcub, hsnc, rv);
}

// ML: MATLAB semantics (WiFi_channel_estimation_*.m): pilot LS averaged over
// blocks 0..3 -- Linear/Cubic/Sinc are linear in the pilot values, so the
// 4-block average of the per-block estimates is the per-block formula applied
// to the averaged pilots -- proper conj in LT_LS, cubic divisors 14/28/42.
// LIGHT: the request is a subset of LT_LS | PS_Linear (BASELINE configs[1]);
// the Cubic/Sinc constants and paths compile out, which keeps the kernel under
// 128 VGPRs (4 waves/SIMD: twice the loads in flight of the generic kernel).
constexpr int LS_PIPE_FRAMES = 4;   // LIGHT: frames per group, the next group's loads issued before this group's math
template <bool EQ, bool ML, bool LIGHT = false>
__global__ __launch_bounds__(256) void ls_kernel(const State *__restrict__ st, LsArgs a)
{
    constexpr bool PIPE = LIGHT;
    constexpr int F = PIPE ? LS_PIPE_FRAMES : LS_FRAMES;   // frames per wave iteration
    const int lane = threadIdx.x & 63;
    const int64_t nw = (int64_t)gridDim.x * LS_WAVES;
    const bool act = lane < NSC;
    const int k = act ? lane : 0;
    const LsLane c = ls_lane(st, a.tx_pre, k);
    const uint32_t mask = LIGHT ? (a.mask & (WCE_EST_LT_LS | WCE_EST_PS_LINEAR)) : a.mask;
    const bool need_lt = (mask & (WCE_EST_LT_LS | WCE_EQUALIZE)) != 0;
    const bool need_ps = (mask & (WCE_EST_PS_LINEAR | WCE_EST_PS_CUBIC | WCE_EST_PS_SINC | WCE_EQUALIZE)) != 0;
    const int pp = lane & 3;
    const int pil = pp == 0 ? WCE_P0 : pp == 1 ? WCE_P1 : pp == 2 ? WCE_P2 : WCE_P3;
    // lanes loading pilots: 4 (one block) or 16 (lane = 4 b + pilot, blocks 0..3)
    const bool pil_lane = ML ? lane < 16 : lane < 4;
    const int64_t pil_off = ML ? (int64_t)(lane >> 2) * a.bs + pil : (int64_t)a.blk * a.bs + pil;
    const bool rx_pre = need_lt && a.rx_pre;

    // every load of F frames, issued before any use
    auto load = [&](int64_t f0, double2 (&ptx)[F], double2 (&prx)[F], double2 (&rp)[F]) {
#pragma unroll
        for (int u = 0; u < F; ++u) {
            const int64_t f = f0 + u < a.n ? f0 + u : a.n - 1;
            ptx[u] = make_double2(1, 0);
            prx[u] = make_double2(0, 0);
            if (need_ps && pil_lane) {
                ptx[u] = ld2(a.tx, f * a.fs + pil_off);
                prx[u] = ld2(a.rx, f * a.fs + pil_off);
            }
            rp[u] = rx_pre ? ld2(a.rx_pre, f * a.ps + k) : make_double2(0, 0);
        }
    };
    const int64_t step = nw * F;
    int64_t f0 = ((int64_t)blockIdx.x * LS_WAVES + (threadIdx.x >> 6)) * F;
    double2 ptx[F], prx[F], rp[F];
    if (f0 < a.n) load(f0, ptx, prx, rp);
    for (; f0 < a.n; f0 += step) {
        double2 ntx[F], nrx[F], nrp[F];
        if (PIPE && f0 + step < a.n) load(f0 + step, ntx, nrx, nrp);   // in flight during this group's math
#pragma unroll
        for (int u = 0; u < F; ++u) {
            const int64_t f = f0 + u;
            if (f >= a.n) break;
            double2 h0 = make_double2(0, 0), h1 = h0, h2 = h0, h3 = h0;
            if (need_ps) {
                double2 hp = cdiv(prx[u], ptx[u]);                       // main.c:82-84
                if (ML) {                                                 // mean over blocks 0..3
                    hp = cadd(hp, shfl_xor_c(hp, 4));
                    hp = cadd(hp, shfl_xor_c(hp, 8));
                    hp = cscale(hp, 0.25);
                }
                h0 = shfl_c(hp, 0); h1 = shfl_c(hp, 1); h2 = shfl_c(hp, 2); h3 = shfl_c(hp, 3);
            }
            const double2 hlt = lt_ls_lane<ML>(c, rx_pre, rp[u], k);
            double2 hlin, hcub, hsnc;
            ps_lane<ML>(c, mask, h0, h1, h2, h3, hlin, hcub, hsnc);
            if (act) ls_store<EQ>(a, f, k, mask, hlt, hlin, hcub, hsnc);
        }
        if (PIPE) {
#pragma unroll
            for (int u = 0; u < F; ++u) { ptx[u] = ntx[u]; prx[u] = nrx[u]; rp[u] = nrp[u]; }
        } else if (f0 + step < a.n) {
            load(f0 + step, ptx, prx, rp);
        }
    }
}

// =====================================================================
// LT_LS + PS_Linear, C semantics (BASELINE configs[1]): ls_elem_kernel below,
// one (frame, subcarrier) element per thread.  The flat-index machinery here
// (frames per launch, 512-element wave-chunks) also serves the REF read-out
// (mmse_ref_flat_kernel) and the non-finite scan.  (Round 1's ls_flat_kernel,
// 512-element chunks per wave, was retired in round 4: profiles/r02_ab_ls.txt.)
// =====================================================================
constexpr int FLAT_U = 8;                               // elements per lane per chunk
constexpr int FLAT_CHUNK = 64 * FLAT_U;                 // 512
constexpr int FLAT_FR = (FLAT_CHUNK - 1) / NSC + 2;     // frames one chunk can touch: 11
static_assert(4 * FLAT_FR <= 64, "one pilot per lane");
// REF PS_MMSE: batches past this many frames (~the 256 MiB MALL at the 1,360 B
// a frame's pilot sectors and H move) run mmse_ref_elem_kernel
constexpr int64_t REF_ELEM_FROM = 196608;
constexpr int64_t FLAT_MAX_FRAMES = 1ll << 26;          // per launch: e < 2^32
// frames per launch of the flat kernels: FLAT_MAX_FRAMES, or a smaller
// multiple of 32 set by wce_debug_set_flat_chunk so that tests reach the
// multi-launch path (f_begin > 0) at sizes a test can afford
static int64_t g_flat_chunk = FLAT_MAX_FRAMES;
static inline int64_t flat_chunk() { return __atomic_load_n(&g_flat_chunk, __ATOMIC_RELAXED); }
int set_flat_chunk(int64_t frames)
{
    if (frames == 0) frames = FLAT_MAX_FRAMES;
    if (frames < 32 || frames > FLAT_MAX_FRAMES || frames % 32) return WCE_EINVAL;
    __atomic_store_n(&g_flat_chunk, frames, __ATOMIC_RELAXED);
    return WCE_OK;
}

// One (frame, subcarrier) element per thread, no grid stride (round 2): the
// store pattern that streams fastest on MI355X (7.0 TB/s one-shot against
// 4.7 TB/s grid-strided, profiles/r02_ubench_hbm.txt).  Each lane loads the
// two pilot pairs its linear segment needs (the lanes of a wave cover ~1.2
// frames, so one pilot load instruction touches ~2 sectors) and divides them
// itself; the arithmetic is ls_kernel's, so outputs are bit-identical.
__global__ __launch_bounds__(256) void ls_elem_kernel(const State *__restrict__ st, LsArgs a, int64_t f_begin,
                                                      uint32_t nfr)
{
    __shared__ double2 s_txp[64], s_hlt[64];
    if (threadIdx.x < NSC) {
        s_txp[threadIdx.x] = ld2(a.tx_pre ? a.tx_pre : st->tx_pre, threadIdx.x);
        s_hlt[threadIdx.x] = ld2(st->h_lt, threadIdx.x);
    }
    __syncthreads();
    const uint32_t e = blockIdx.x * 256u + threadIdx.x;
    if (e >= nfr * (uint32_t)NSC) return;
    const uint32_t f = e / NSC, k = e - f * NSC;
    const bool do_lt = (a.mask & WCE_EST_LT_LS) && a.lt, do_lin = (a.mask & WCE_EST_PS_LINEAR) && a.lin;
    const bool f32 = a.f32 != 0;
    const int64_t fg = f_begin + f;
    const int seg = k < WCE_P1 ? 0 : (k < WCE_P2 ? 1 : 2);
    double2 plo_t = make_double2(1, 0), plo_r = make_double2(0, 0), phi_t = plo_t, phi_r = plo_r, rp = plo_r;
    if (do_lin) {
        const int64_t o = fg * a.fs + (int64_t)a.blk * a.bs;
        const int plo = seg == 0 ? WCE_P0 : (seg == 1 ? WCE_P1 : WCE_P2);
        const int phi = seg == 0 ? WCE_P1 : (seg == 1 ? WCE_P2 : WCE_P3);
        plo_t = ld2(a.tx, o + plo);   // (cached: the next frame's lanes reuse the sectors; nontemporal 588 -> 625 us)
        plo_r = ld2(a.rx, o + plo);
        phi_t = ld2(a.tx, o + phi);
        phi_r = ld2(a.rx, o + phi);
    }
    if (do_lt && a.rx_pre) {
        rp = ld2_nt(a.rx_pre, fg * a.ps + k);   // streamed once: nontemporal
    }
    const int64_t out = fg * a.os + k;
    if (do_lt) {                                    // main.c:66-75
        double2 h = s_hlt[k];
        if (a.rx_pre) {
            const double2 t = s_txp[k];
            const double cq = t.x - t.y;
            h = cdiv(make_double2(cq * rp.x, cq * rp.y), make_double2(cq * t.x, cq * t.y));
        }
        if (k == WCE_DC) h = make_double2(0, 0);
        st_out(a.lt, out, h, f32);
    }
    if (do_lin) {                                   // main.c:82-99
        const double alpha = (double)((int)k - (seg == 0 ? WCE_P0 : (seg == 1 ? WCE_P1 : WCE_P2))) * (1.0 / 14.0);
        const double2 lo = cdiv(plo_r, plo_t), hi = cdiv(phi_r, phi_t);
        st_out(a.lin, out, clerp(lo, hi, alpha), f32);
    }
}

// =====================================================================
// PS_MMSE in REF (main.c) semantics: a = 0, so Ryy = 2 ow2 I is diagonal and
// X keeps the 4 pilots only (main.c:148-212, repaired as in DESIGN.md s2):
// H_f = u_f s_f with s_f = sum_p w_f[P_p] tx_f[P_p] rx_f[P_p] / b.  Per frame
// that is 4 pilot pairs in (64-B sectors, as the LS path) and 53 outputs:
// HBM-bound, so it runs over the flat element index e = 53 f + k -- lanes 4j+p
// form frame j's pilot terms, a quad DPP sum gives s_j into a per-wave LDS
// table, and every element lane writes u[k] s.  cs == 0: one shared (u, w)
// (the ctx's C_ref); cs != 0: per-frame factors (WCE_MMSE_FRAME_COV).
// =====================================================================
template <int CTRL>
__device__ __forceinline__ double dpp_quad(double v)
{
    const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xf, 0xf, true);   // quad_perm: every lane has a
    const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xf, 0xf, true);   // source, no old value needed
    return __hiloint2double(hi, lo);
}
// sum over the 4 lanes of each quad, ((t0 + t1) + (t2 + t3)) in every lane
__device__ __forceinline__ double2 quad_sum_c(double2 t)
{
    t = cadd(t, make_double2(dpp_quad<0xB1>(t.x), dpp_quad<0xB1>(t.y)));   // quad_perm [1,0,3,2]
    return cadd(t, make_double2(dpp_quad<0x4E>(t.x), dpp_quad<0x4E>(t.y)));  // quad_perm [2,3,0,1]
}

// REF pilot term w x r and the output u s, with contraction off: every REF
// kernel (flat, tiles, and the config-4 element kernel) rounds them alike
// whatever code surrounds them, so their outputs stay bit-identical.
__device__ __forceinline__ double2 ref_term(double2 w, double2 x, double2 r)
{
#pragma clang fp contract(off)
    const double2 c = make_double2(w.x * x.x - w.y * x.y, w.x * x.y + w.y * x.x);
    return make_double2(c.x * r.x - c.y * r.y, c.x * r.y + c.y * r.x);
}
__device__ __forceinline__ double2 ref_sum4(double2 t0, double2 t1, double2 t2, double2 t3, double rb)
{
#pragma clang fp contract(off)
    const double2 a = make_double2(t0.x + t1.x, t0.y + t1.y), b = make_double2(t2.x + t3.x, t2.y + t3.y);
    return make_double2((a.x + b.x) * rb, (a.y + b.y) * rb);
}
__device__ __forceinline__ double2 ref_out(double2 u, double2 s)
{
#pragma clang fp contract(off)
    return make_double2(u.x * s.x - u.y * s.y, u.x * s.y + u.y * s.x);
}

__global__ __launch_bounds__(256) void mmse_ref_flat_kernel(const State *__restrict__ st, SolveArgs a, int64_t f_begin,
                                                            uint32_t nfr)
{
    __shared__ double2 s_u[64];
    __shared__ double2 s_s[LS_WAVES][FLAT_FR];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const bool shared = a.cs == 0;
    if (shared && threadIdx.x < NSC) s_u[threadIdx.x] = ld2(a.cu, threadIdx.x);
    __syncthreads();
    const double rb = 1.0 / st->bcoef;
    const uint32_t E = nfr * (uint32_t)NSC;
    const uint32_t nchunks = (E + FLAT_CHUNK - 1) / FLAT_CHUNK;
    const int pj = lane & 3;
    const int pil = pj == 0 ? WCE_P0 : pj == 1 ? WCE_P1 : pj == 2 ? WCE_P2 : WCE_P3;
    double2 *s_tab = s_s[w];
    for (uint32_t c = blockIdx.x * LS_WAVES + w; c < nchunks; c += gridDim.x * LS_WAVES) {
        const uint32_t e0 = c * FLAT_CHUNK;
        const uint32_t ff = e0 / NSC;
        // ---- loads: pilot terms (lanes 4j+p) and, per frame, the u rows
        double2 xt = make_double2(0, 0), xr = xt, wp = xt;
        const uint32_t fr = min(ff + (uint32_t)(lane >> 2), nfr - 1);
        if (lane < 4 * FLAT_FR) {
            const int64_t o = (f_begin + fr) * a.fs + (int64_t)a.blk * a.bs + pil;
            xt = ld2(a.tx, o);
            xr = ld2(a.rx, o);
            const int64_t wo = shared ? pil : (f_begin + fr) * a.cs + pil;
            wp = a.cw ? ld2(a.cw, wo) : cconj(ld2(a.cu, wo));
        }
        double2 uf[FLAT_U];
        if (!shared) {
#pragma unroll
            for (int i = 0; i < FLAT_U; ++i) {
                const uint32_t e = min(e0 + 64u * i + lane, E - 1);
                const uint32_t f = e / NSC, k = e - f * NSC;
                uf[i] = ld2(a.cu, (f_begin + f) * a.cs + k);
            }
        }
        const double2 sj = quad_sum_c(ref_term(wp, xt, xr));   // w^T X rx over frame j's pilots
        if (lane < 4 * FLAT_FR && pj == 0) s_tab[lane >> 2] = ref_sum4(sj, make_double2(0, 0), make_double2(0, 0),
                                                                      make_double2(0, 0), rb);
        wave_lds_sync();
#pragma unroll
        for (int i = 0; i < FLAT_U; ++i) {
            const uint32_t e = e0 + 64u * i + lane;
            const uint32_t f = e / NSC, k = e - f * NSC;
            const int jl = (int)(f - ff) < FLAT_FR ? (int)(f - ff) : FLAT_FR - 1;
            const double2 u = shared ? s_u[k] : uf[i];
            if (e < E) st2(a.w, (f_begin + f) * a.ws + k, ref_out(u, s_tab[jl]));
        }
        wave_lds_sync();   // s_tab is rewritten by the next chunk
    }
}

// The same read-out with one (frame, subcarrier) element per thread and no
// grid stride (round 6; ls_elem_kernel's store pattern), for batches past the
// MALL.  A wave's 64 consecutive elements touch at most 3 frames: lanes 4j+p
// (j < 3) load frame ff + j's pilot pair p -- issued before the block's u
// staging, so the two latencies overlap -- the same quad DPP sum forms s_j,
// and each lane takes its frame's s from lane 4j by readlane (no LDS round
// trip, no chunk loop: the hardware keeps many such short waves in flight).
// Arithmetic and summation order are mmse_ref_flat_kernel's: outputs
// bit-identical.  Measured (1,048,576 frames, profiles/r06_ab_ref_elem.txt):
// 381 -> 337 us against the capped chunks; 2 or 4 elements per lane (462, 440),
// plain stores (371), 128 / 512 / 1,024-thread blocks (375 / 340 / 365) lose, and
// an XCD-aware block remap (each XCD one contiguous run) changes nothing (342),
// and neither does one frame per wave (344 vs 343: no frame's pilot sectors
// fetched by two waves, so that re-fetch is not what holds it).
__global__ __launch_bounds__(256) void mmse_ref_elem_kernel(const State *__restrict__ st, SolveArgs a, int64_t f_begin,
                                                            uint32_t nfr)
{
    __shared__ double2 s_u[64];
    const int lane = threadIdx.x & 63;
    const bool shared = a.cs == 0;
    const uint32_t E = nfr * (uint32_t)NSC;
    const uint32_t e0 = blockIdx.x * 256u + (threadIdx.x & ~63u);     // the wave's first element
    const uint32_t ff = min(e0 / NSC, nfr - 1);
    const int pj = lane & 3;
    const int pil = pj == 0 ? WCE_P0 : pj == 1 ? WCE_P1 : pj == 2 ? WCE_P2 : WCE_P3;
    double2 xt = make_double2(0, 0), xr = xt, wp = xt, uf = xt;
    if (lane < 12) {
        const uint32_t fr = min(ff + (uint32_t)(lane >> 2), nfr - 1);
        const int64_t o = (f_begin + fr) * a.fs + (int64_t)a.blk * a.bs + pil;
        xt = ld2(a.tx, o);
        xr = ld2(a.rx, o);
        const int64_t wo = shared ? pil : (f_begin + fr) * a.cs + pil;
        wp = a.cw ? ld2(a.cw, wo) : cconj(ld2(a.cu, wo));
    }
    const uint32_t e = e0 + lane;
    const uint32_t f = min(e / NSC, nfr - 1), k = e - f * NSC;
    if (!shared && e < E) uf = ld2(a.cu, (f_begin + f) * a.cs + k);
    if (shared && threadIdx.x < NSC) s_u[threadIdx.x] = ld2(a.cu, threadIdx.x);
    __syncthreads();
    const double rb = 1.0 / st->bcoef;
    const double2 sj = ref_sum4(quad_sum_c(ref_term(wp, xt, xr)), make_double2(0, 0), make_double2(0, 0),
                                make_double2(0, 0), rb);
    double sr[3], si[3];
#pragma unroll
    for (int j = 0; j < 3; ++j) {
        sr[j] = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(sj.x), 4 * j),
                                 __builtin_amdgcn_readlane(__double2loint(sj.x), 4 * j));
        si[j] = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(sj.y), 4 * j),
                                 __builtin_amdgcn_readlane(__double2loint(sj.y), 4 * j));
    }
    const uint32_t j = f - ff;
    const double2 s = make_double2(j == 0 ? sr[0] : j == 1 ? sr[1] : sr[2], j == 0 ? si[0] : j == 1 ? si[1] : si[2]);
    if (e < E) st2_nt(a.w, (f_begin + f) * a.ws + k, ref_out(shared ? s_u[k] : uf, s));
}

// =====================================================================
// BASELINE configs[4] in main.c semantics (round 3): REF PS_MMSE with any of
// LT_LS / PS_Linear / PS_Cubic / PS_Sinc and equalization, one pass over HBM
// (main.c:66-212, WiFi_Equalization.m:1-9).  REF has no factorisation (Ryy =
// 2 ow2 I), so the whole request is streaming: one (frame, subcarrier) element
// per thread, no grid stride (ls_elem_kernel's store pattern).  Each thread
// gathers its frame's 4 pilot pairs (the ~1.2 frames a wave covers share their
// 64-B sectors, so a pilot load instruction touches ~2 of them) and serves
// every output of its element from them: the pilot LS values h_p (main.c:
// 82-84) feed PS_Linear/Cubic/Sinc, s = w^T X rx / b (over the same pilots)
// gives H_MMSE = u s, rx_pre its LT_LS, and the 15 rx blocks of its subcarrier
// (all loads issued before any use) the equalized symbols.  The arithmetic is
// ls_kernel's (ls_lane / lt_ls_lane / ps_lane / ls_store_rv) and
// mmse_ref_flat_kernel's (quad order ((t0 + t1) + (t2 + t3)) * (1 / b)), so the
// outputs are bit-identical to the separate passes.  a.cs != 0: per-frame
// factors u_f, w_f (WCE_MMSE_FRAME_COV).
// =====================================================================
template <bool EQ>
__global__ __launch_bounds__(256) void ref_ls_elem_kernel(const State *__restrict__ st, SolveArgs a, LsArgs l,
                                                          int64_t f_begin, uint32_t nfr)
{
    const uint32_t e = blockIdx.x * 256u + threadIdx.x;
    if (e >= nfr * (uint32_t)NSC) return;
    const uint32_t fl = e / NSC;
    const int k = (int)(e - fl * NSC);
    const int64_t f = f_begin + fl;
    const bool shared = a.cs == 0;
    // ---- every load first
    const int64_t po = f * a.fs + (int64_t)a.blk * a.bs;
    const bool mm = !a.mmse_done;   // REF frame covariance: ref_fc_kernel wrote H already
    double2 xt[4], xr[4], wp[4] = {};
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        xt[p] = ld2(a.tx, po + PILOT[p]);
        xr[p] = ld2(a.rx, po + PILOT[p]);
        const int64_t wo = shared ? PILOT[p] : f * a.cs + PILOT[p];
        if (mm) wp[p] = a.cw ? ld2(a.cw, wo) : cconj(ld2(a.cu, wo));
    }
    const double2 uk = mm ? ld2(a.cu, shared ? k : f * a.cs + k) : make_double2(0, 0);
    const double2 rp = l.rx_pre ? ld2_nt(l.rx_pre, f * l.ps + k) : make_double2(0, 0);
    double2 rv[NBLK];
    if constexpr (EQ) {
#pragma unroll
        for (int b = 0; b < NBLK; b++) rv[b] = ld2_nt(l.rx, f * l.fs + k + b * l.bs);
    }
    const LsLane c = ls_lane(st, l.tx_pre, k);
    // ---- PS_MMSE (REF): H = u s, s = w^T X rx / b over the 4 pilots
    if (mm) {
        double2 tp[4];
#pragma unroll
        for (int p = 0; p < 4; ++p) tp[p] = ref_term(wp[p], xt[p], xr[p]);
        st2(a.w, f * a.ws + k, ref_out(uk, ref_sum4(tp[0], tp[1], tp[2], tp[3], 1.0 / st->bcoef)));
    }
    // ---- LS family + equalization
    double2 h[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) h[p] = cdiv(xr[p], xt[p]);                 // main.c:82-84
    const double2 hlt = lt_ls_lane<false>(c, l.rx_pre != nullptr, rp, k);
    double2 hlin, hcub, hsnc;
    ps_lane<false>(c, l.mask, h[0], h[1], h[2], h[3], hlin, hcub, hsnc);
    ls_store_rv<EQ>(l, f, k, l.mask, hlt, hlin, hcub, hsnc, rv);
}

// =====================================================================
// MMSE solve.  One wave per frame, lane = 8p + q holds A[p+8a][q+8b] for the
// 28 register blocks a >= b (a, b < 7): the block-cyclic 8x8 grid spreads the
// shrinking trailing matrix evenly over lanes.  Row 53 holds conj(rx), so the
// factorisation of [[Ryy, rx], [rx', *]] also runs the forward solve.
//
// Cholesky (Ryy = L L'): pivot k publishes c_k = u_k / sqrt(d_k) (one
// v_rsq_f64 and a third-order refinement step, rsq_nr / rsq_lane), so both
// rank-1 operands are read as published.  Each 8-column panel runs row-per-lane
// (chol_panel: lane l holds A[l][8 KB + c], one full-wave store publishes the
// pivot column, in-panel operands by DPP64 row_newbcast); the trailing blocks
// stay block-cyclic.  One-step lookahead: the column holding k + 1 is updated
// first, the next pivot formed and published to the other half of a ping-pong
// LDS buffer, then the bulk of step k is issued, hiding the pivot chain and the
// LDS round trip.  Dead lanes (upper halves of diagonal blocks, padding row
// 55, panel rows above the pivot) are off in EXEC for their FMAs (cmsub_live):
// the kernels run at the board's power cap, and the saved lane energy is clock.
// (Round 1's square-root-free LDL' on the block-cyclic grid was retired in
// round 4; DESIGN.md s5 has the measurements.)
// =====================================================================
constexpr int RB = 7;     // 7 x 8 = 56 >= 54 rows
typedef double v4d __attribute__((ext_vector_type(4)));   // one v_mfma_f64_16x16x4 accumulator
constexpr int KSTEPS = 14;   // 4-deep MFMA k-steps over 56 >= 53 subcarriers

constexpr int CVS = 9;    // row stride (complex) of the panel transpose buffer

// R0 > 0 (the Gram path at K0 >= 2, rows 8 K0 .. 55 only): the panel transpose
// buffer holds rows R0 .. 55, so the wave needs less LDS and more waves fit a CU.
template <int R0>
struct SolveLdsT {
    static constexpr int ROW0 = R0;
    static constexpr bool TAP_MAPS = false;   // TapsLds: the tap <-> column maps stay in LDS
    __device__ int ci(int row, int c) const { return (row - R0) * CVS + c; }   // conv element (row, c)
    double2 u[2][64];     // pivot column k (unscaled A[:, k]) ping-pong
    double2 x[64];        // masked tx of the frame (diagonal of X), 0 past 53
    double2 rx[64];
    union {
        struct {
            double2 blk[64];  // diagonal 8x8 block of u during back-substitution
            double2 z[64];    // solution
            double rd[64];    // r_k = 1 / d_k, 0 past 52
        };
        double2 conv[(56 - R0) * CVS];   // row-per-lane panels: block column -> rows (to_rows)
        struct {                  // the tap-domain Gram's DFT pair tables (dft_pairs), past blk / z / rd
            double2 pad_bzr[160];
            double2 pa[32], pb[32];   // c_k + c_{53-k}, c_k - c_{53-k}, k = 1..26 (complex vectors)
            double2 rp[32];           // the same for the real vector |x|^2, {sum, difference}
        } tp;
    };
};
using SolveLds = SolveLdsT<0>;
static_assert(sizeof(SolveLds::tp.pad_bzr) == 2 * sizeof(SolveLds::blk) + sizeof(SolveLds::rd),
              "the tap pair tables start past blk / z / rd");
// The tap-domain kernel at K0 = 0: the tap <-> column maps, s_j and E are
// loaded with the frame (one memory round trip instead of three serialized
// ones); the maps stay in LDS past the factorisation.  E stays in
// SolveLds::u[0] until the factorisation reuses it and is reloaded for the
// read-out: keeping it too (13,184 B per wave) measured 2.6% slower, the
// maps alone 1.6% faster (profiles/r05_ab_taps.txt).
struct TapsLds : SolveLds {
    static constexpr bool TAP_MAPS = true;
    uint8_t tap[64], col[64];   // State::tap_of / col_of (col 0xff: no column)
};
static_assert(sizeof(TapsLds) == 12288, "12 waves of the tap kernel per CU");
// conv element (row, c) at (row - R0) * 9 + c (SolveLdsT::ci): the odd row
// stride keeps both the block-cyclic stores and the row reads bank-conflict
// free (an XOR swizzle of an unpadded buffer measured 1% slower: address VALU).



// acc -= l conj(c) on the lanes of the (compile-time) lane mask m only.  The
// other lanes carry elements that are never read (upper halves of diagonal
// blocks, padding row 55, rows above the pivot in a row panel).  Their FMAs
// are switched off in EXEC for the four FMAs (and
// EXEC restored) inside one asm statement: written as a C++ branch the
// compiler turns it into selects and divergent control flow that spills.
// The masked lanes keep their old (dead) values: "+v" ties in to out.
__device__ __forceinline__ void cmsub_live(uint64_t m, double2 &acc, double2 l, double2 c)
{
    if (m != ~0ull) {
        // m & EXEC is formed by the compiler: the asm itself writes no SCC
        // (an s_and_b64 in here would clobber an SCC live across it)
        const uint64_t em = m & __builtin_amdgcn_read_exec();
        uint64_t sv;
        asm("s_mov_b64 %[sv], exec\n\t"
            "s_mov_b64 exec, %[m]\n\t"
            "v_fma_f64 %[ax], -%[lx], %[cx], %[ax]\n\t"
            "v_fma_f64 %[ax], -%[ly], %[cy], %[ax]\n\t"
            "v_fma_f64 %[ay], -%[ly], %[cx], %[ay]\n\t"
            "v_fma_f64 %[ay], %[lx], %[cy], %[ay]\n\t"
            "s_mov_b64 exec, %[sv]"
            : [ax] "+v"(acc.x), [ay] "+v"(acc.y), [sv] "=&s"(sv)
            : [lx] "v"(l.x), [ly] "v"(l.y), [cx] "v"(c.x), [cy] "v"(c.y), [m] "s"(em));
    } else {
        cmsub_conj(acc, l, c);
    }
}
// compile-time lane masks (lane = 8p + q)
constexpr uint64_t lanes_from(int lo, int hi)   // lanes lo..hi
{
    uint64_t m = 0;
    for (int l = lo; l <= hi && l < 64; ++l) m |= 1ull << l;
    return m;
}
constexpr uint64_t lanes_lower(int qmin)   // q <= p, p < 7, q > qmin
{
    uint64_t m = 0;
    for (int p = 0; p < 7; ++p)
        for (int q = qmin + 1; q <= p; ++q) m |= 1ull << (8 * p + q);
    return m;
}
constexpr uint64_t kRows55 = lanes_from(0, 55);   // p < 7: block row 6 without padding row 55

// Trailing block column BB: the diagonal block keeps its lower triangle
// (q <= p; in block 6 that includes the (54, 53) corner), and block row 6
// has no row 55 (p < 7).  cm: lanes whose column is still live (all but the
// LDL lookahead's own block column).
constexpr uint64_t kLower = lanes_lower(-1) | ~kRows55;   // q <= p, block rows 0..5
template <int BB>
__device__ __forceinline__ void upd_col_live(double2 (&A)[RB][RB], const double2 (&Ur)[RB], double2 v, uint64_t cm = ~0ull)
{
    if constexpr (BB == RB - 1) {
        cmsub_live(cm & lanes_lower(-1), A[BB][BB], Ur[BB], v);
    } else {
        cmsub_live(cm & kLower, A[BB][BB], Ur[BB], v);
#pragma unroll
        for (int aa = BB + 1; aa < RB - 1; ++aa) cmsub_live(cm, A[aa][BB], Ur[aa], v);
        cmsub_live(cm & kRows55, A[RB - 1][BB], Ur[RB - 1], v);
    }
}
// 1/sqrt(d) of the pivot d that lane L holds, as a wave-uniform scalar.  The
// kernel is power-capped, so the 6-op chain runs on lane L alone (EXEC = that
// lane inside the asm, ANDed with the incoming EXEC so that a switched-off lane
// is never written) and comes back through v_readlane: the same arithmetic as
// rsq_nr (one third-order step after v_rsq_f64), bit-identical, at 1/64 of its
// energy.  L is a constant after unrolling and every caller runs on the full
// wave.  (Rounds 2-5 read d out to an SGPR first and ran the chain on the
// lowest active lane: two more v_readlane per pivot; round 6, 470 -> 454 us per
// 65,536 frames, profiles/r06_ab_rsq_lane.txt.)
__device__ __forceinline__ double rsq_lane(double dv, int L)
{
    double y, t, e;
    uint64_t sv;
    const double c38 = 0.375;
    asm("s_mov_b64 %[sv], exec\n\t"
        "s_mov_b64 exec, %[m]\n\t"
        "v_rsq_f64 %[y], %[d]\n\t"
        "s_nop 1\n\t"
        "v_mul_f64 %[t], %[d], %[y]\n\t"
        "v_fma_f64 %[e], -%[t], %[y], 1.0\n\t"
        "v_mul_f64 %[t], %[y], %[e]\n\t"
        "v_fma_f64 %[e], %[e], %[c], 0.5\n\t"
        "v_fma_f64 %[y], %[t], %[e], %[y]\n\t"
        "s_mov_b64 exec, %[sv]"
        : [y] "=&v"(y), [t] "=&v"(t), [e] "=&v"(e), [sv] "=&s"(sv)
        : [d] "v"(dv), [c] "s"(c38), [m] "s"((1ull << L) & __builtin_amdgcn_read_exec()));
    return readlane_f64(y, L);
}

// (Round 1's block-cyclic square-root-free LDL^H -- ldl_step / ldl_panel, a
// masked 8-lane publish per pivot -- was retired in round 4; every path runs
// the Cholesky row panels below.  Its measurements: profiles/r01_ab_publish.txt,
// r02_ab_dense.txt.)

// ---------------------------------------------------------------------
// Row-per-lane panels (the rank-1 read-out path, DOT).  Publishing pivot
// column k+1 from the block-cyclic grid takes 7 - KB masked ds_write_b128 per
// step (8 owner lanes each); an LDS store costs its issuing SIMD far more than
// its 16 B suggest (profiles/r01_ab_publish.txt).  So panel KB (block column KB = columns
// 8KB .. 8KB+7, every row) is held transposed: lane l holds P[c] = A[l][8KB+c].
// Column k+1 is then ONE register across the wave and goes out in one
// full-wave store.  In-panel updates P[c] -= (r_k P[kq]) conj(A[8KB+c][k])
// take the wave-uniform operand from the published column (LDS broadcast);
// the trailing blocks aa >= bb > KB stay block-cyclic as before.  At a panel's
// last step block column KB+1 is updated, written once to LDS by all lanes and
// read back transposed (6 - KB stores + 8 reads per panel).
// ---------------------------------------------------------------------
template <int KB, typename L = SolveLds>
__device__ __forceinline__ void to_rows(const double2 (&A)[RB][RB], double2 (&P)[8], L &s, int p, int q,
                                        int lane)
{
#pragma unroll
    for (int aa = KB; aa < RB; ++aa) s.conv[s.ci(p + 8 * aa, q)] = A[aa][KB];
    wave_lds_sync();
    int l = lane < 56 ? lane : 55;   // lanes 56..63 carry a copy of row 55 (never read)
    l = l < L::ROW0 ? L::ROW0 : l;   // (R0 > 0: rows above the system read row R0; never read either)
#pragma unroll
    for (int c = 0; c < 8; ++c) P[c] = s.conv[s.ci(l, c)];
}

// Back-substitution L' z = w (unit diagonal), rows 8*BLK .. 8*BLK+7.  The
// registers hold u = L D; r_j = 1/d_j rescales sums once per column.
template <int N>
__device__ __forceinline__ double2 bcast_lane_c(double2 w)
{
    double2 z;
    asm volatile("s_nop 1\n\t"
                 "v_mov_b64_dpp %[zx], %[wx] row_newbcast:%c[n] row_mask:0xf bank_mask:0xf\n\t"
                 "v_mov_b64_dpp %[zy], %[wy] row_newbcast:%c[n] row_mask:0xf bank_mask:0xf"
                 : [zx] "=&v"(z.x), [zy] "=&v"(z.y)
                 : [wx] "v"(w.x), [wy] "v"(w.y), [n] "i"(N));
    return z;
}
// lane t (< NMAX) of every 16-lane row, to all lanes (t a constant after unrolling)
template <int NMAX>
__device__ __forceinline__ double2 bcast_row_lane(double2 w, int t)
{
    switch (t) {
    case 0: return bcast_lane_c<0>(w);
    case 1: return bcast_lane_c<1>(w);
    case 2: return bcast_lane_c<2>(w);
    case 3: return bcast_lane_c<3>(w);
    case 4: return bcast_lane_c<4>(w);
    case 5: return bcast_lane_c<5>(w);
    case 6: return bcast_lane_c<6>(w);
    default: return bcast_lane_c<7>(w);
    }
}

template <int BLK, typename L = SolveLds>
__device__ __forceinline__ void back_block(const double2 (&A)[RB][RB], double2 (&P)[RB], const double (&rq)[RB],
                                           L &s, int p, int q, int lane)
{
    constexpr int NROW = (BLK == RB - 1) ? (NSC - 8 * (RB - 1)) : 8;
    // w_j = r_j * (conj(u_53,j) - sum_{i solved} conj(u_ij) z_i),  j = 8*BLK + q
    double2 w = P[BLK];
    w = sum_over_p(w);   // DPP + permlane swaps: no LDS traffic
    w = cscale(w, rq[BLK]);
    // L = u r of the diagonal block, strictly lower part only, scaled and
    // masked once by its owner (r depends on the column q only)
    s.blk[lane] = (q < p) ? cscale(A[BLK][BLK], rq[BLK]) : make_double2(0.0, 0.0);
    wave_lds_sync();
    // lb[t] = L[8*BLK + t][8*BLK + q] for q < t, else 0: a lane's w_q is left
    // untouched once row q is solved, so it ends holding z_q
    double2 lb[NROW];
#pragma unroll
    for (int t = 0; t < NROW; ++t) lb[t] = s.blk[8 * t + q];
#pragma unroll
    for (int t = NROW - 1; t >= 0; --t) {
        // every lane with q = t holds w_t = z_t; DPP row_newbcast:t hands lane t
        // of each 16-lane row to the whole row (two VALU movs instead of four
        // readlanes through SGPRs; s_nop 1: w was written by the previous row)
        const double2 z = bcast_row_lane<8>(w, t);
        cmsub_conj(w, z, lb[t]);                               // w_q -= conj(L[i][q]) z_i, q < t
    }
    if (p == 0 && q < NROW) s.z[8 * BLK + q] = w;              // one store per block
    wave_lds_sync();
    const double2 zp = s.z[8 * BLK + p];                       // rows >= 53 read 0
#pragma unroll
    for (int bb = 0; bb < BLK; ++bb) cmsub_conj(P[bb], zp, A[BLK][bb]);
}

constexpr int SOLVE_WAVES_PER_SIMD = 3;   // the per-frame solve kernels (rank-1 and dense C)
// Dense C, scaled form.  Ryy = a X C X^H + b I = a X M X^H with
// M = C + diag(b / (a |x_i|^2)), so Ryy^-1 rx = X^-H M^-1 y / a, y = X^-1 rx,
// and W = X z = (x / (a conj x)) o (M^-1 y).  M is C itself off the diagonal:
// the build is the 28 block loads and a diagonal add, instead of two complex
// products per element.  Cholesky's accuracy is invariant under the diagonal
// scaling X (van der Sluis), so this is the same solve.  A subcarrier with
// x_i = 0 (or a |x_i|^2 < 1e-200 b) leaves Ryy's row i as b e_i and W_i = 0:
// it gets y_i = 0 and M_ii = 1e200, whose coupling |C_ij|^2 / M_ii is below
// half an ulp of every other entry, and phase 0.
constexpr double kDenseMaskedDiag = 1e200;
// (written so that a NaN |x|^2 counts as kept: non-finite input stays non-finite in H, where the guard sees it)
__device__ __forceinline__ bool dense_keep(double tt, double bc) { return !(tt <= 0.0 || tt * 1e200 <= bc); }
// One block's solve; returns w_lane = x_lane z_lane (0 for lanes >= 53 is
// not guaranteed: callers store lanes < 53 only).
// FC: per-frame rank-1 covariance C_f = cu_f cw_f^T (SolveArgs::cu/cw, frame f)
// instead of the shared State::C.
// DOT (rank-1 C = u w^T only): a second bordered row 54 = (w o x)^T rides in
// the padding lanes of register row 6.  Eliminating pivots 0..52 then leaves
// the Schur complement -w^T X Ryy^-1 rx in element (54, 53), so H = u s with
// s = w^T X z needs neither the back-substitution nor the C W product; the
// function returns s (wave-uniform) instead of x_lane z_lane.
// ---------------------------------------------------------------------
// Cholesky form of the row panels (default).  Publishing c_k = u_k / sqrt(d_k)
// instead of u_k makes the rank-1 term symmetric, A -= c c^H: both operands
// are read from the one published column as they are -- no per-block scaling
// of the column operand (2 (6 - KB) MULs per step) and no r_k u_k for the
// panel.  The price is 1/sqrt instead of 1/d (3 more VALU per step).
// ---------------------------------------------------------------------
template <int BB>
__device__ __forceinline__ void upd_col_chol(double2 (&A)[RB][RB], const double2 (&Ur)[RB], double2 v, int p, int q)
{
    upd_col_live<BB>(A, Ur, v);
}

template <int BB>
__device__ __forceinline__ void upd_cols_chol(double2 (&A)[RB][RB], const double2 (&Ur)[RB], const double2 *col, int p,
                                              int q)
{
    if constexpr (BB < RB) {
        upd_col_chol<BB>(A, Ur, col[q + 8 * BB], p, q);
        upd_cols_chol<BB + 1>(A, Ur, col, p, q);
    }
}

// acc -= l conj(c_k[8KB + N]) for the row-per-lane panel, where R holds
// c_k[8KB + (lane & 7)]: DPP row_newbcast:N hands lane N of each 16-lane row
// (= c_k[8KB + N]) to the whole row as the FMA's first operand (gfx950's
// DPP64 on v_fmac_f64), so the 7 - kq wave-uniform operands of a step cost
// one LDS read instead of one each.  row_mask RM switches off the 16-lane
// rows that hold no live row (all lanes < 8KB + N).  R comes straight from a
// ds_read, so the "VALU writes VGPR -> DPP reads it: 2 wait states" hazard
// cannot arise unless the compiler copies R with a VALU move just before;
// tests/test_isa.py checks the compiled code for exactly that.
template <int N, int RM>
__device__ __forceinline__ void cmsub_bc(double2 &acc, double2 l, double2 R)
{
    asm("v_fmac_f64_dpp %[ax], -%[cx], %[lx] row_newbcast:%c[n] row_mask:%c[rm] bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %[ax], -%[cy], %[ly] row_newbcast:%c[n] row_mask:%c[rm] bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %[ay], -%[cx], %[ly] row_newbcast:%c[n] row_mask:%c[rm] bank_mask:0xf\n\t"
        "v_fmac_f64_dpp %[ay], %[cy], %[lx] row_newbcast:%c[n] row_mask:%c[rm] bank_mask:0xf"
        : [ax] "+v"(acc.x), [ay] "+v"(acc.y)
        : [lx] "v"(l.x), [ly] "v"(l.y), [cx] "v"(R.x), [cy] "v"(R.y), [n] "i"(N), [rm] "i"(RM));
}
constexpr int live_rows(int first) { return 0xf & ~((1 << (first / 16)) - 1); }   // 16-lane rows holding lanes >= first
template <int KB>
__device__ __forceinline__ void cmsub_panel(int c, double2 &acc, double2 l, double2 R)
{
    switch (c) {   // c is a constant after unrolling: one case survives
    case 1: cmsub_bc<1, live_rows(8 * KB + 1)>(acc, l, R); break;
    case 2: cmsub_bc<2, live_rows(8 * KB + 2)>(acc, l, R); break;
    case 3: cmsub_bc<3, live_rows(8 * KB + 3)>(acc, l, R); break;
    case 4: cmsub_bc<4, live_rows(8 * KB + 4)>(acc, l, R); break;
    case 5: cmsub_bc<5, live_rows(8 * KB + 5)>(acc, l, R); break;
    case 6: cmsub_bc<6, live_rows(8 * KB + 6)>(acc, l, R); break;
    default: cmsub_bc<7, live_rows(8 * KB + 7)>(acc, l, R); break;
    }
}

// Panel KB in row form.  Entering: P = block column KB with P[0] = c_{8KB}
// (scaled), c_{8KB} published.
// K0 = 1: pivot 8KB is already eliminated (exact_first_step), c_{8KB+1} published.
// R: c_k[8KB + (lane & 7)] for the step about to run, read
// for step k+1 right after c_{k+1} is published, so the next lookahead does
// not wait for an LDS round trip.
// rsel = sel ? rs : rsel, materialised now: left to itself the compiler
// sinks the chain of selects to the end and keeps every pivot's rs alive
__device__ __forceinline__ void keep_rsel(double &rsel, bool sel, double rs)
{
    rsel = sel ? rs : rsel;
    asm volatile("" : "+v"(rsel));
}

// a = c where sel (component selects on values: a select between an A
// element and a temporary as lvalues would defeat SROA and put A in scratch)
__device__ __forceinline__ void keep_where(bool sel, double2 &a, double2 c)
{
    a.x = sel ? c.x : a.x;
    a.y = sel ? c.y : a.y;
}

// rsel[lane L] = rs (wave-uniform, in SGPRs): one v_mov_b64 under EXEC = lane L
// instead of v_cmp + two v_cndmask per step.  L is a constant after unrolling.
// The mask is ANDed with the incoming EXEC (formed outside the asm, which
// writes no SCC), so a lane switched off around the call is never written.
__device__ __forceinline__ void keep_rsel_lane(double &rsel, int L, double rs)
{
    uint64_t sv;
    asm volatile("s_mov_b64 %[sv], exec\n\t"
                 "s_mov_b64 exec, %[m]\n\t"
                 "v_mov_b64 %[r], %[v]\n\t"
                 "s_mov_b64 exec, %[sv]"
                 : [r] "+v"(rsel), [sv] "=&s"(sv)
                 : [m] "s"((1ull << L) & __builtin_amdgcn_read_exec()), [v] "s"(rs));
}
constexpr uint64_t lanes_q(int qq) { return 0x0101010101010101ull << qq; }   // lanes with q == qq

// KEEP (the dense-C path, which back-substitutes): every finished panel is
// written back into its block column of A (to_blocks), block column 6 keeps
// its scaled columns, and rsel collects 1/sqrt(d_k) in lane k.
// Column c of a finished panel goes to conv as soon as it is final (after its
// own step's in-panel updates, stash_col), so the panel's registers free up
// column by column; to_blocks then only reads the block column back.
template <typename L = SolveLds>
__device__ __forceinline__ void stash_col(L &s, int lane, int c, double2 v)
{
    if (lane < 56 && lane >= L::ROW0) s.conv[s.ci(lane, c)] = v;
}
template <int KB, typename L = SolveLds>
__device__ __forceinline__ void to_blocks(double2 (&A)[RB][RB], const double2 (&P)[8], L &s, int p, int q,
                                          int lane)
{
    stash_col(s, lane, 7, P[7]);
    wave_lds_sync();
#pragma unroll
    for (int aa = KB; aa < RB; ++aa) A[aa][KB] = s.conv[s.ci(p + 8 * aa, q)];
    wave_lds_sync();   // to_rows<KB + 1> reuses conv
}

template <int KB, int K0 = 0, bool KEEP = false, typename L = SolveLds>
__device__ __forceinline__ void chol_panel(double2 (&A)[RB][RB], double2 (&P)[8], double2 &R, L &s, int p,
                                           int q, int lane, double &rsel)
{
#pragma unroll
    for (int kq = K0; kq < 8; ++kq) {
        const int k = 8 * KB + kq;
        const double2 *col = s.u[k & 1];
        double2 *next = s.u[(k + 1) & 1];
        double2 Ur[RB];
#pragma unroll
        for (int aa = KB + 1; aa < RB; ++aa) Ur[aa] = col[p + 8 * aa];
        if (kq < 7) {
            // row lane of column 8KB+c is live for 8KB+c <= lane <= 54
            cmsub_panel<KB>(kq + 1, P[kq + 1], P[kq], R);   // lookahead
            const double rs = rsq_lane(P[kq + 1].x, k + 1);
            P[kq + 1] = cscale(P[kq + 1], rs);
            next[lane] = P[kq + 1];                               // publish c_{k+1}: one store
            if (KEEP) keep_rsel_lane(rsel, k + 1, rs);
            wave_lds_sync();
            const double2 Rn = next[8 * KB + (lane & 7)];
#pragma unroll
            for (int c = kq + 2; c < 8; ++c) {
                cmsub_panel<KB>(c, P[c], P[kq], R);
            }
            if (KEEP) stash_col(s, lane, kq, P[kq]);   // final: its last use was above
            upd_cols_chol<KB + 1>(A, Ur, col, p, q);
            R = Rn;
        } else {
            upd_col_chol<KB + 1>(A, Ur, col[q + 8 * (KB + 1)], p, q);
            if (KEEP) to_blocks<KB>(A, P, s, p, q, lane);
            if constexpr (KB + 2 < RB) {
                to_rows<KB + 1>(A, P, s, p, q, lane);
                const double rs = rsq_lane(P[0].x, k + 1);
                P[0] = cscale(P[0], rs);
                next[lane] = P[0];
                if (KEEP) keep_rsel_lane(rsel, k + 1, rs);
                wave_lds_sync();
                R = next[8 * (KB + 1) + (lane & 7)];
            } else {   // block column 6 stays block-cyclic: the 8 owners of column 48 publish
                const double rs = rsq_lane(A[KB + 1][KB + 1].x, 0);
                const double2 cs = cscale(A[KB + 1][KB + 1], rs);
                if (q == 0) next[p + 8 * (KB + 1)] = cs;
                if (KEEP) {
                    keep_rsel_lane(rsel, k + 1, rs);
                    keep_where_mask(lanes_q(0), q == 0, A[KB + 1][KB + 1], cs);
                }
            }
            upd_cols_chol<KB + 2>(A, Ur, col, p, q);
        }
        wave_lds_sync();
    }
}

// Pivots 48..52 on register block (6, 6) and the read-out.  Eliminated
// columns take unmasked updates (never read again); (54, 53) receives every
// step, the last (pivot 52) straight from the published c_52.
template <typename L = SolveLds>
__device__ __forceinline__ double2 chol_last(double2 (&A)[RB][RB], L &s, int p, int q)
{
    constexpr int B6 = 8 * (RB - 1);
#pragma unroll
    for (int kq = 0; kq < NSC - 1 - B6; ++kq) {
        const int k = B6 + kq;
        const double2 *col = s.u[k & 1];
        double2 *next = s.u[(k + 1) & 1];
        cmsub_live(lanes_lower(kq), A[RB - 1][RB - 1], col[p + B6], col[q + B6]);
        const double rs = rsq_lane(A[RB - 1][RB - 1].x, 9 * (kq + 1));
        const double2 cs = cscale(A[RB - 1][RB - 1], rs);
        if (q == kq + 1) next[p + B6] = cs;
        wave_lds_sync();
    }
    const double2 *col = s.u[(NSC - 1) & 1];   // c_52
    double2 sc = readlane_c(A[RB - 1][RB - 1], 8 * (NSC + 1 - B6) + (NSC - B6));   // (54, 53)
    cmsub_conj(sc, col[NSC + 1], col[NSC]);
    return make_double2(-sc.x, -sc.y);   // s = -S(54, 53)
}

// Pivots 49..52 on register block (6, 6) keeping L (the dense-C path):
// each finished column is scaled in place (lanes q == kq), rsel collects
// 1/sqrt(d).  Entering: column 48 scaled in place and published.
template <typename L = SolveLds>
__device__ __forceinline__ void chol_last_keep(double2 (&A)[RB][RB], L &s, int p, int q, int lane, double &rsel)
{
    constexpr int B6 = 8 * (RB - 1);
#pragma unroll
    for (int kq = 0; kq < NSC - 1 - B6; ++kq) {
        const int k = B6 + kq;
        const double2 *col = s.u[k & 1];
        double2 *next = s.u[(k + 1) & 1];
        cmsub_live(lanes_lower(kq), A[RB - 1][RB - 1], col[p + B6], col[q + B6]);
        const double rs = rsq_lane(A[RB - 1][RB - 1].x, 9 * (kq + 1));
        const double2 cs = cscale(A[RB - 1][RB - 1], rs);
        if (q == kq + 1) next[p + B6] = cs;
        keep_rsel_lane(rsel, k + 1, rs);
        keep_where_mask(lanes_q(kq + 1), q == kq + 1, A[RB - 1][RB - 1], cs);
        wave_lds_sync();
    }
}

template <int KB, typename L = SolveLds>
__device__ __forceinline__ void chol_panels_keep(double2 (&A)[RB][RB], double2 (&P)[8], double2 &R, L &s,
                                                 int p, int q, int lane, double &rsel)
{
    if constexpr (KB < RB - 1) {
        chol_panel<KB, 0, true>(A, P, R, s, p, q, lane, rsel);
        chol_panels_keep<KB + 1>(A, P, R, s, p, q, lane, rsel);
    }
}

// The dense-C factorisation: the headline's row-per-lane
// Cholesky panels on Ryy bordered by conj(rx) (row 53), keeping L in the
// block-cyclic registers for the back-substitution; s.rd = 1/sqrt(d_k).
// Entering: A built (block rows/columns K0..6, row 53 = the conj right-hand
// side).  K0 > 0 (the low-rank path, mmse_lr_kernel): the system occupies
// rows 8 K0 .. 52 only and the panels before it are skipped.
template <int K0 = 0, typename L = SolveLds>
__device__ __forceinline__ void dense_chol(double2 (&A)[RB][RB], L &s, int p, int q, int lane)
{
    double rsel = 0.0;
    if constexpr (K0 < RB - 1) {
        double2 P[8];
        to_rows<K0>(A, P, s, p, q, lane);
        if constexpr (K0 > 0) {   // rows above the system: defined values (updated, never read)
#pragma unroll
            for (int c = 0; c < 8; ++c) keep_where(lane < 8 * K0, P[c], make_double2(0.0, 0.0));
        }
        const double r0 = rsq_nr(readlane_f64(P[0].x, 8 * K0));
        rsel = lane == 8 * K0 ? r0 : 0.0;
        P[0] = cscale(P[0], r0);
        wave_lds_sync();   // conv reads done before the publish (s.u is separate; order only)
        s.u[0][lane] = P[0];
        wave_lds_sync();
        double2 R = s.u[0][8 * K0 + (lane & 7)];
        chol_panels_keep<K0>(A, P, R, s, p, q, lane, rsel);
    } else {   // the system is block (6, 6) alone: pivot 48 opens the block-cyclic last panel
        const double rs = rsq_lane(A[RB - 1][RB - 1].x, 0);
        const double2 cs = cscale(A[RB - 1][RB - 1], rs);
        if (q == 0) s.u[0][p + 8 * (RB - 1)] = cs;
        keep_rsel_lane(rsel, 8 * (RB - 1), rs);
        keep_where_mask(lanes_q(0), q == 0, A[RB - 1][RB - 1], cs);
        wave_lds_sync();
    }
    chol_last_keep(A, s, p, q, lane, rsel);
    wave_lds_sync();
    s.rd[lane] = lane < NSC ? rsel : 0.0;   // conv is dead: rd and z share its LDS
    s.z[lane] = make_double2(0.0, 0.0);     // rows >= 53 must read 0 in the back-substitution
    wave_lds_sync();
}

// ---------------------------------------------------------------------
// Exact first elimination step (the rank-1 read-out path).  Ryy = al be^T + b I
// with al = a x o u, be = w o conj(x) = conj(al) / a (w = conj(u) whenever
// a != 0).  Its cond is 1 + |al|^2 / b ~ 4e6 on the synthetic frames: rounding
// the entries al_i be_j to fp64 alone perturbs s = (w o x)^T Ryy^-1 rx by up to
// ~1e-10 norm-relative, and a plain fp64 factorisation reaches 1.7e-9 on frames
// whose channel is unrelated to the preamble's (profiles/r01_accuracy_probe.txt).
// All of that ill-conditioning is consumed by the first pivot: eliminating
// pivot m leaves
//     S_ij = al_i be_j (b / d0) + b [i == j],   d0 = al_m be_m + b,
// whose rank-1 part is at most 52 b when m is the largest |al_m| (cond <= 53).
// So S is formed directly from the factors -- never as the fp64 difference
// al_i be_j - (al_i be_m)(al_m be_j) / d0 -- and so are the two bordered rows:
//     row 53: conj(rx_j) - conj(rx_m) al_m be_j / d0
//     row 54: rho_j - rho_m al_m be_j / d0 = w_j [x_j b/d0 + kap/d0 x_m (conj(x_m) x_j - x_m conj(x_j))]
//             (rho = w o x, kap = a w_m u_m; the bracket has no cancellation)
//     (54, 53): -rho_m rx_m / d0.
// Pivot m is swapped with index 0 (s is invariant under a symmetric
// permutation); index 0 then holds b on the diagonal and zeros elsewhere, so
// the factorisation proper runs over pivots 1..52 of the 53 x 53 matrix.
// LDS out: u[0] = al' (scaled by b/d0), u[1] = be', z = rx', blk = rho' and
// blk[53] = the (54, 53) entry; all permuted, index 0 zero.
// ---------------------------------------------------------------------
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v)
{
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, m, 64));
    return v;
}

template <typename L = SolveLds>
__device__ __forceinline__ void exact_first_step(const SolveArgs &a, L &s, int64_t f, double ac, double bc)
{
    const int lane = threadIdx.x;
    const bool act = lane < NSC;
    const double2 uf = act ? ld2(a.cu, f * a.cs + lane) : make_double2(0, 0);
    const double2 wf = !act ? make_double2(0, 0) : a.cw ? ld2(a.cw, f * a.cs + lane) : cconj(uf);
    const double2 xl = s.x[lane];
    const double2 rxl = s.rx[lane];
    const double2 al = cscale(cmul(xl, uf), ac);
    const double2 be = cmul(wf, cconj(xl));
    // pivot: the largest |al_l|^2 (float key, lane in the low 6 bits; ties and
    // the last few mantissa bits do not matter for the choice)
    const float mag = (float)(al.x * al.x + al.y * al.y);
    const uint32_t key = act ? ((__float_as_uint(mag) & ~63u) | (uint32_t)lane) : 0u;
    const int m = __builtin_amdgcn_readfirstlane((int)(wave_max_u32(key) & 63u));
    const double2 alm = readlane_c(al, m), bem = readlane_c(be, m);
    const double2 xm = readlane_c(xl, m), rxm = readlane_c(rxl, m);
    const double2 um = readlane_c(uf, m), wm = readlane_c(wf, m);
    const double d0 = (alm.x * bem.x - alm.y * bem.y) + bc;
    const double r0 = rcp_nr(d0);
    const double sc = bc * r0;
    // row 53: rx'_l = rx_l - rx_m conj(al_m be_l) / d0
    const double2 rxp = csub(rxl, cscale(cmul(rxm, cconj(cmul(alm, be))), r0));
    // row 54: w_l [x_l b/d0 + (kap/d0) x_m 2i Im(conj(x_m) x_l)]
    const double ti = 2.0 * (xm.x * xl.y - xm.y * xl.x);
    const double2 kr = cscale(cmul(make_double2(ac * wm.x, ac * wm.y), um), r0);
    const double2 ixm = make_double2(-xm.y * ti, xm.x * ti);   // x_m 2i Im(.)
    double2 rhop = cmul(wf, cadd(cscale(xl, sc), cmul(kr, ixm)));
    double2 alp = cscale(al, sc), bep = be, rxo = rxp;
    if (lane == m) alp = bep = rxo = rhop = make_double2(0, 0);
    if (lane == NSC) {   // the (54, 53) entry: -rho_m rx_m / d0
        const double2 rhom = cmul(wm, xm);
        rhop = cscale(cmul(rhom, rxm), -r0);
    }
    const int dst = lane == m ? 0 : (lane == 0 ? m : lane);
    s.u[0][dst] = alp;
    s.u[1][dst] = bep;
    s.z[dst] = rxo;
    s.blk[dst] = rhop;
}

// The rank-1 read-out path (a != 0): Ryy = a (x o u)(w o x')^T + b I bordered
// by conj(rx) (row 53) and (w o x)^T (row 54), factorised with row-per-lane
// Cholesky panels 0..5 (chol_panel) and the block-cyclic last panel
// (chol_last); returns s = -S(54, 53) = w^T X Ryy^-1 rx.
template <typename L = SolveLds>
__device__ __forceinline__ double2 dot_factor(const State *__restrict__ st, const SolveArgs &a, L &s,
                                              int64_t f, double ac, double bc)
{
    const int lane = threadIdx.x;
    const int p = lane >> 3, q = lane & 7;
    exact_first_step(a, s, f, ac, bc);
    wave_lds_sync();
    double2 A[RB][RB];
    double2 P[8];
    {   // panel 0 in rows: P[c] = a x_l u_l w_c conj(x_c) + b [l == c]
        const double2 ul = s.u[0][lane];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            P[c] = cmul(ul, s.u[1][c]);
            P[c].x += (lane == c) ? bc : 0.0;
        }
        if (lane == NSC) {
#pragma unroll
            for (int c = 0; c < 8; ++c) P[c] = cconj(s.z[c]);
        }
        if (lane == NSC + 1) {
#pragma unroll
            for (int c = 0; c < 8; ++c) P[c] = s.blk[c];
        }
    }
    // trailing blocks aa >= bb >= 1, block-cyclic
#pragma unroll
    for (int aa = 1; aa < RB; ++aa)
#pragma unroll
        for (int bb = 1; bb <= aa; ++bb) A[aa][bb] = cmul(s.u[0][p + 8 * aa], s.u[1][q + 8 * bb]);
    const double bdiag = (p == q) ? bc : 0.0;
#pragma unroll
    for (int aa = 1; aa < RB - 1; ++aa) A[aa][aa].x += bdiag;
    A[RB - 1][RB - 1].x += (p == q && p < NSC - 8 * (RB - 1)) ? bc : 0.0;
    if (p == NSC - 8 * (RB - 1)) {   // row 53 = conj(rx'), rx after the exact first step
#pragma unroll
        for (int bb = 1; bb < RB; ++bb) A[RB - 1][bb] = cconj(s.z[q + 8 * bb]);
    }
    if (p == NSC + 1 - 8 * (RB - 1)) {   // row 54 = (w o x)^T
#pragma unroll
        for (int bb = 1; bb < RB; ++bb) A[RB - 1][bb] = s.blk[q + 8 * bb];
    }
    wave_lds_sync();   // s.u[0] is reused by the first publish
    // pivot 0 was eliminated exactly (column 0 is b e_0): the
    // factorisation starts at pivot 1, whose column the build left final
    P[1] = cscale(P[1], rsq_nr(readlane_f64(P[1].x, 1)));
    s.u[1][lane] = P[1];
    wave_lds_sync();
    double2 R = s.u[1][lane & 7];
    double rsel = 0.0;   // unused (no back-substitution)
    chol_panel<0, 1>(A, P, R, s, p, q, lane, rsel);
    chol_panel<1>(A, P, R, s, p, q, lane, rsel);
    chol_panel<2>(A, P, R, s, p, q, lane, rsel);
    chol_panel<3>(A, P, R, s, p, q, lane, rsel);
    chol_panel<4>(A, P, R, s, p, q, lane, rsel);
    chol_panel<5>(A, P, R, s, p, q, lane, rsel);
    return chol_last(A, s, p, q);
}

template <bool FC, bool DOT = false, typename L = SolveLds>
__device__ __forceinline__ double2 solve_block(const State *__restrict__ st, const SolveArgs &a, L &s,
                                               int64_t base, int64_t f)
{
    const int lane = threadIdx.x;
    const int p = lane >> 3, q = lane & 7;
    const double ac = st->acoef, bc = st->bcoef;
    double2 A[RB][RB];
    const bool cbuild = !FC && ac != 0.0;
    if constexpr (!DOT && !FC) {   // dense C: its 28 block loads in the frame's round trip
        if (cbuild) {             // (M = C + diag(b / (a |x|^2)); C zero-padded: no bounds checks)
#pragma unroll
            for (int aa = 0; aa < RB; ++aa)
#pragma unroll
                for (int bb = 0; bb <= aa; ++bb) A[aa][bb] = ld2(st->C, (p + 8 * aa) * CLD + q + 8 * bb);
        }
    }
    {
        const bool act = lane < NSC;
        // branch-free: both loads issued together (and with C's: one memory round trip
        // where the dense path waited three, 655.7 -> 644.7 us, profiles/r05_ab_dense_early.txt)
        const int lc = act ? lane : NSC - 1;
        const double2 t0 = ld2(a.tx, base + lc), r0 = ld2(a.rx, base + lc);
        const double2 t = act ? t0 : make_double2(0, 0);
        const double2 r = act ? r0 : make_double2(0, 0);
        const bool inx = act && ((st->xmask >> lane) & 1ull);
        s.x[lane] = inx ? t : make_double2(0, 0);
        s.rx[lane] = r;
        s.z[lane] = make_double2(0, 0);
        s.rd[lane] = 0.0;
        if (!DOT && cbuild) {   // y = rx / x to u[0], M's diagonal to u[1] (read by the build)
            const double2 xl = inx ? t : make_double2(0, 0);
            const double tt = ac * (xl.x * xl.x + xl.y * xl.y);
            const bool keep = dense_keep(tt, bc);
            const double inv = keep ? 1.0 / tt : 0.0;
            s.u[0][lane] = cscale(cmul(r, cconj(xl)), ac * inv);
            s.u[1][lane] = make_double2(keep ? bc * inv : kDenseMaskedDiag, 0.0);
        }
    }
    wave_lds_sync();
    if constexpr (DOT) {
        if (ac == 0.0) {   // REF (main.c): Ryy = 2 ow2 I is diagonal, z = rx / b -- no factorisation
            const bool act = lane < NSC;
            const double2 uf = act ? ld2(a.cu, f * a.cs + lane) : make_double2(0, 0);
            const double2 wf = !act ? make_double2(0, 0) : a.cw ? ld2(a.cw, f * a.cs + lane) : cconj(uf);
            double2 t = act ? cmul(cmul(wf, s.x[lane]), s.rx[lane]) : make_double2(0, 0);
#pragma unroll
            for (int m = 32; m >= 1; m >>= 1) t = cadd(t, shfl_xor_c(t, m));
            return cscale(t, 1.0 / bc);   // s = w^T X rx / b
        }
        return dot_factor(st, a, s, f, ac, bc);
    }
    {
        if (FC && ac != 0.0) {   // a X u w^T X': both factors staged in the pivot buffers
            const bool act = lane < NSC;
            const double2 uf = act ? ld2(a.cu, f * a.cs + lane) : make_double2(0, 0);
            const double2 wf = !act ? make_double2(0, 0) : a.cw ? ld2(a.cw, f * a.cs + lane) : cconj(uf);
            const double2 xl = s.x[lane];
            s.u[0][lane] = cscale(cmul(xl, uf), ac);
            s.u[1][lane] = cmul(wf, cconj(xl));
            wave_lds_sync();
#pragma unroll
            for (int aa = 0; aa < RB; ++aa)
#pragma unroll
                for (int bb = 0; bb <= aa; ++bb) A[aa][bb] = cmul(s.u[0][p + 8 * aa], s.u[1][q + 8 * bb]);
            wave_lds_sync();   // the factorisation reuses s.u[0]
        } else if (cbuild) {   // M = C + diag(b / (a |x|^2)): C loaded with the frame (above)
        } else {
#pragma unroll
            for (int aa = 0; aa < RB; ++aa)
#pragma unroll
                for (int bb = 0; bb <= aa; ++bb) A[aa][bb] = make_double2(0, 0);
        }
        // scaled dense form: M's diagonal from u[1], bordered row conj(y) from u[0]
        const bool scaled = cbuild;
        const double2 *brow = scaled ? s.u[0] : s.rx;
#pragma unroll
        for (int aa = 0; aa < RB - 1; ++aa) A[aa][aa].x += (p == q) ? (scaled ? s.u[1][p + 8 * aa].x : bc) : 0.0;
        A[RB - 1][RB - 1].x += (p == q && p < NSC - 8 * (RB - 1)) ? (scaled ? s.u[1][p + 8 * (RB - 1)].x : bc) : 0.0;
        // bordered row 53 = conj(rx)  (lanes p == 5, register row 6).  A branch, not
        // a select: a select on an A element defeats SROA (A would live in scratch).
        if (p == NSC - 8 * (RB - 1)) {
#pragma unroll
            for (int bb = 0; bb < RB; ++bb) A[RB - 1][bb] = cconj(brow[q + 8 * bb]);
        }
    }
    dense_chol(A, s, p, q, lane);
    wave_lds_sync();
    // row 53 holds conj(u_53,j) = conj(y_j): w_j = r_j conj(u_53,j)
    double rq[RB];
#pragma unroll
    for (int bb = 0; bb < RB; ++bb) rq[bb] = s.rd[q + 8 * bb];
    double2 P[RB];
    const bool brow = (p == NSC - 8 * (RB - 1));
#pragma unroll
    for (int bb = 0; bb < RB; ++bb) P[bb] = brow ? cconj(A[RB - 1][bb]) : make_double2(0, 0);
    back_block<6>(A, P, rq, s, p, q, lane);
    back_block<5>(A, P, rq, s, p, q, lane);
    back_block<4>(A, P, rq, s, p, q, lane);
    back_block<3>(A, P, rq, s, p, q, lane);
    back_block<2>(A, P, rq, s, p, q, lane);
    back_block<1>(A, P, rq, s, p, q, lane);
    back_block<0>(A, P, rq, s, p, q, lane);
    wave_lds_sync();
    const double2 xl = s.x[lane];
    if (cbuild) {   // W = (x / (a conj x)) o (M^-1 y)
        const double tt = ac * (xl.x * xl.x + xl.y * xl.y);
        const double2 ph = dense_keep(tt, bc) ? cscale(cmul(xl, xl), 1.0 / tt) : make_double2(0.0, 0.0);
        return cmul(ph, s.z[lane]);
    }
    return cmul(xl, s.z[lane]);
}

// R1: Ryy built from the rank-1 factors SolveArgs::cu/cw (TEXTBOOK: State::cvec)
// instead of the dense State::C (COV mode, or a = 0).
// split (MATLAB averaging): one wave per (frame, block), W_b to row g of a.w.
template <bool R1>
__global__ __launch_bounds__(64, SOLVE_WAVES_PER_SIMD) void mmse_solve_kernel(const State *__restrict__ st, SolveArgs a)
{
    __shared__ SolveLds s;
    const int64_t g = blockIdx.x;
    const int64_t f = a.split ? g / a.nblk : g;
    const int b = a.split ? (int)(g - f * a.nblk) : 0;
    if (f >= a.n || (a.skip && a.skip[g])) return;   // skip: H already written (constant-modulus path)
    const double2 w = solve_block<R1>(st, a, s, f * a.fs + (int64_t)(a.blk + b) * a.bs, f);
    if (threadIdx.x < NSC) st2(a.w, g * a.ws + threadIdx.x, w);
}

// =====================================================================
// WCE_MMSE_COV, low-rank path (round 3).  C = U U^H with U = F V_r
// sqrt(Lambda_r) (State::U, r columns, from the 80-bit eigendecomposition of
// Rhh in wce_state.cpp).  With G = X U (53 x r):
//     H = C X Ryy^-1 rx = U s,   s = U^H X Ryy^-1 rx,   Ryy = a G G^H + b I,
// and by the push-through identity G^H (a G G^H + b I)^-1 = (a G^H G + b I)^-1 G^H
//     s = t = (a G^H G + b I_r)^-1 G^H rx                      (real x),
// while for complex x (U^H X = U^H X^H + U^H (X - X^H), b Ryy^-1 rx = rx - a G t)
//     s = t + U^H [(x - conj x) o (rx - a x o (U t))] / b.
// The dense form (mmse_solve_kernel: z = Ryy^-1 rx, then C X z) carries the
// components of z along C's null space, of size |rx|/b, which C X must
// cancel: it loses ~eps cond(Ryy) on a rank-deficient C, 2e-10 .. 1e-8 here
// (DESIGN.md s2).  This form never creates them: the error stays at the
// 1e-13 level for every rank (profiles/r03_accuracy_probe.txt).
//
// The r x r Gram system reuses the dense solve's machinery: it is embedded
// in the block-cyclic registers at block row K0 = (53 - r) / 8 (rows 8 K0 ..
// 8 K0 + r - 1; rows up to 52 past r get Gram entries 0, i.e. pivot b and a
// zero right-hand side, so t_j = 0 there), bordered by conj(G^H rx) in row 53
// exactly where the dense solve keeps conj(rx); the panels before K0 and
// their back-substitution blocks are skipped.  G^H G and the border row are
// accumulated on the VALU from G~ = [X U | rx] staged through LDS (the border
// is the Gram column j = 53 - 8 K0 of G~; lr_gram_valu).  (Round 3's MFMA
// Gram tiles, 1.25-1.33x slower, were retired in round 4:
// profiles/r03_ab_lowrank_dense.txt.)
// =====================================================================
constexpr int LR_WAVES_PER_SIMD = 4;   // K0 >= 2 (<= 122 VGPRs); 12 KB of LDS per wave caps a CU at 13 waves anyway
// Gram column j of G~ at subcarrier k: x_k U[k][j] (U is zero past column
// r - 1), rx_k at the border column j = 53 - 8 K0, 0 past it.
template <int K0, typename L = SolveLds>
__device__ __forceinline__ double2 lr_gcol(const State *__restrict__ st, const L &s, int k, int j)
{
    constexpr int RMAX = NSC - 8 * K0;
    const double2 g = cmul(s.x[k], ld2(st->U, k * CLD + j));   // k, j < 64 (U zero-padded)
    const double2 r = j == RMAX ? s.rx[k] : make_double2(0.0, 0.0);
    return j < RMAX ? g : r;
}
// The Gram blocks on the VALU, straight into the block-cyclic layout:
// G~ is staged through LDS 8 subcarriers at a time (T[kk][j], j < 56 - 8 K0),
// and lane (p, q) accumulates A[aa][bb] += conj(G~[k][p + 8 (aa - K0)])
// G~[k][q + 8 (bb - K0)] for its blocks aa >= bb >= K0 only -- no upper
// tiles, no padding columns, 4 FMAs per element and subcarrier, where the
// MFMA tiles execute ~2-4x that (16 x 16 tiles over 56 - 8 K0 rows, both
// triangles, 4 real MFMAs per complex product).  Operand reads: lanes that
// share p (or q) read one address, so each ds_read_b128 touches <= 8 slots.
constexpr int LR_KC = 8;   // subcarriers per staged chunk
template <int K0, typename L = SolveLds>
__device__ __forceinline__ void lr_gram_valu(const State *__restrict__ st, L &s, double2 (&A)[RB][RB],
                                             int lane, int p, int q, double ac, double bc)
{
    constexpr int NC = 8 * (RB - K0);   // staged Gram columns (block rows K0..6)
    constexpr int NB = RB - K0;
    static_assert(LR_KC * NC <= (56 - L::ROW0) * CVS, "chunk fits the conv buffer");
    double2 *T = s.conv;
#pragma unroll
    for (int aa = K0; aa < RB; ++aa)
#pragma unroll
        for (int bb = K0; bb <= aa; ++bb) A[aa][bb] = make_double2(0.0, 0.0);
#pragma unroll 1
    for (int k0 = 0; k0 < 56; k0 += LR_KC) {
#pragma unroll
        for (int e = lane; e < LR_KC * NC; e += 64) {
            const int kk = e / NC, j = e - kk * NC;
            T[e] = lr_gcol<K0>(st, s, k0 + kk, j);
        }
        wave_lds_sync();
#pragma unroll 2
        for (int kk = 0; kk < LR_KC; ++kk) {
            double2 rw[NB], cl[NB];
#pragma unroll
            for (int m = 0; m < NB; ++m) {
                rw[m] = T[kk * NC + p + 8 * m];
                cl[m] = T[kk * NC + q + 8 * m];
            }
#pragma unroll
            for (int m = 0; m < NB; ++m)
#pragma unroll
                for (int n = 0; n <= m; ++n) {   // += conj(rw) cl
                    double2 &acc = A[K0 + m][K0 + n];
                    acc.x = fma(rw[m].x, cl[n].x, fma(rw[m].y, cl[n].y, acc.x));
                    acc.y = fma(rw[m].x, cl[n].y, fma(-rw[m].y, cl[n].x, acc.y));
                }
        }
        wave_lds_sync();   // the next chunk rewrites T
    }
#pragma unroll
    for (int aa = K0; aa < RB; ++aa) {
        const bool gram = p + 8 * aa < NSC;   // rows 53 (border), 54, 55 stay as they are
#pragma unroll
        for (int bb = K0; bb <= aa; ++bb) {
            double2 e = cscale(A[aa][bb], ac);
            e.x += (gram && aa == bb && p == q) ? bc : 0.0;
            A[aa][bb] = make_double2(gram ? e.x : A[aa][bb].x, gram ? e.y : A[aa][bb].y);
        }
    }
}

template <int BLK, int K0, typename L = SolveLds>
__device__ __forceinline__ void back_blocks_from(const double2 (&A)[RB][RB], double2 (&P)[RB], const double (&rq)[RB],
                                                 L &s, int p, int q, int lane)
{
    if constexpr (BLK >= K0) {
        back_block<BLK>(A, P, rq, s, p, q, lane);
        back_blocks_from<BLK - 1, K0>(A, P, rq, s, p, q, lane);
    }
}

// One (frame, block): returns H_k on lane k (k < 53).
template <int K0, typename L = SolveLds>
__device__ __forceinline__ double2 lr_solve(const State *__restrict__ st, const SolveArgs &a, L &s, int64_t base)
{
    constexpr int RMAX = NSC - 8 * K0;
    const int lane = threadIdx.x;
    const int p = lane >> 3, q = lane & 7;
    const bool act = lane < NSC;
    const double ac = st->acoef, bc = st->bcoef;
    double2 xl;
    {
        const double2 t = act ? ld2(a.tx, base + lane) : make_double2(0, 0);
        const double2 r = act ? ld2(a.rx, base + lane) : make_double2(0, 0);
        const bool inx = act && ((st->xmask >> lane) & 1ull);
        xl = inx ? t : make_double2(0, 0);
        s.x[lane] = xl;
        s.rx[lane] = r;
    }
    wave_lds_sync();
    double2 A[RB][RB];
#pragma unroll
    for (int aa = 0; aa < RB; ++aa)
#pragma unroll
        for (int bb = 0; bb <= aa; ++bb) A[aa][bb] = make_double2(0.0, 0.0);
    lr_gram_valu<K0>(st, s, A, lane, p, q, ac, bc);
    dense_chol<K0>(A, s, p, q, lane);
    double rq[RB];
#pragma unroll
    for (int bb = 0; bb < RB; ++bb) rq[bb] = s.rd[q + 8 * bb];
    double2 P[RB];
    const bool brow = (p == NSC - 8 * (RB - 1));
#pragma unroll
    for (int bb = 0; bb < RB; ++bb) P[bb] = brow ? cconj(A[RB - 1][bb]) : make_double2(0, 0);
    back_blocks_from<RB - 1, K0>(A, P, rq, s, p, q, lane);
    wave_lds_sync();
    // t_j = z[8 K0 + j]; y = U t on lane k (UT rows: coalesced)
    const int r = min(st->cov_rank, RMAX);
    const int kk = act ? lane : 0;
    double2 y = make_double2(0.0, 0.0);
#pragma unroll 4
    for (int j = 0; j < r; ++j) {
        const double2 u = ld2(st->UT, j * CLD + kk), t = s.z[8 * K0 + j];
        y.x = fma(u.x, t.x, fma(-u.y, t.y, y.x));
        y.y = fma(u.x, t.y, fma(u.y, t.x, y.y));
    }
    if (__ballot(act && xl.y != 0.0) != 0) {   // complex symbols: s = t + U^H [(x - conj x) o rho] / b
        const double2 rho = csub(s.rx[lane], cscale(cmul(xl, y), ac));   // b Ryy^-1 rx
        s.blk[lane] = act ? make_double2(-2.0 * xl.y * rho.y, 2.0 * xl.y * rho.x) : make_double2(0, 0);
        wave_lds_sync();
        double2 c = make_double2(0.0, 0.0);   // lane j: c_j = sum_k conj(U[k][j]) v_k
        const int jj = lane < r ? lane : 0;
#pragma unroll 4
        for (int k = 0; k < NSC; ++k) {
            const double2 u = ld2(st->U, k * CLD + jj), v = s.blk[k];
            c.x = fma(u.x, v.x, fma(u.y, v.y, c.x));
            c.y = fma(u.x, v.y, fma(-u.y, v.x, c.y));
        }
        s.u[1][lane] = cscale(c, 1.0 / bc);
        wave_lds_sync();
#pragma unroll 4
        for (int j = 0; j < r; ++j) {
            const double2 u = ld2(st->UT, j * CLD + kk), t = s.u[1][j];
            y.x = fma(u.x, t.x, fma(-u.y, t.y, y.x));
            y.y = fma(u.x, t.y, fma(u.y, t.x, y.y));
        }
    }
    return y;
}

// ---------------------------------------------------------------------
// The tap-domain Gram (State::cov_taps, a diagonal Rhh = power-delay profile).
// U[k][j] = s_j E[k t_j mod 53] (E[m] = exp(-2 pi i m / 53), t_j the tap of
// column j, s_j = sqrt(lambda_j)), so with p = |x|^2 and v = x o conj(rx)
//     (U^H P U)_ij = s_i s_j Q((t_i - t_j) mod 53),  Q(d) = sum_k p_k conj(E[k d])
//     (rx^H X U)_j = s_j D(t_j),                    D(m) = sum_k v_k E[k m]
// -- two 53-point DFTs on lane d / m (6 FMAs per subcarrier), where the
// product Gram runs ~100 per subcarrier per lane at K0 = 0.  The read-out
// y = U t is a third DFT of the tap vector c_t = s_t t_col(t), and the
// complex-symbol correction U U^H v / b the conjugate DFT of v scaled by
// lambda_t, then a fourth.  E[k d mod 53] is gathered from LDS by the exact
// index recurrence (no phase accumulation).
// ---------------------------------------------------------------------
// Every DFT here runs over pairs (k, 53 - k): E[(53 - k) m] = conj(E[k m]), so
//     c_k E[km] + c_{53-k} conj(E[km]) = (c_k + c_{53-k}) Re E[km] + i (c_k - c_{53-k}) Im E[km]
// -- one gather and half the FMAs and index steps of the plain sum.
// pair tables of the LDS vector c (53 complex) on lanes 1..26
__device__ __forceinline__ void dft_pairs(const double2 *c, double2 *pa, double2 *pb, int lane)
{
    if (lane >= 1 && lane <= NSC / 2) {
        const double2 u = c[lane], w = c[NSC - lane];
        pa[lane] = cadd(u, w);
        pb[lane] = csub(u, w);
    }
}
// y(m) = c_0 + sum_k (pa_k Re E[k m] + i pb_k Im E[k m]) over the pairs (k, 53 - k), outputs m and 53 - m together (E[k (53 - m)] =
// conj(E[k m]): A = sum pa_k Re E, B = i sum pb_k Im E (CONJ: -Im), y(m) = c_0 + A
// + B, y(53 - m) = c_0 + A - B), half-wave h over the pairs k = 1 + 13 h ..
// 13 + 13 h; the halves meet in xs (>= 59 entries of free LDS), which ends up
// holding y, returned on lane m (lanes past 52: y(0)).
template <bool CONJ>
__device__ __forceinline__ double2 lr_dft53_split(const double2 *e, const double2 *pa, const double2 *pb, double2 c0,
                                                  int lane, double2 *xs)
{
    const int h = lane >> 5, d = lane & 31;
    const bool dv = d <= NSC / 2;
    const int dd = dv ? d : 0;
    const int k0 = 1 + (NSC / 4) * h;
    const uint32_t st = 16u * (uint32_t)dd, sw = st - 16u * NSC;
    uint32_t o = 16u * (uint32_t)((k0 * dd) % NSC);
    double2 A = make_double2(0.0, 0.0), B = A;
#pragma unroll 2
    for (int j = 0; j < NSC / 4; ++j) {
        const int k = k0 + j;
        const double2 w = ld_e(e, o), va = pa[k], vb = pb[k];
        const double wy = CONJ ? -w.y : w.y;
        A.x = fma(va.x, w.x, A.x);
        A.y = fma(va.y, w.x, A.y);
        B.x = fma(-vb.y, wy, B.x);
        B.y = fma(vb.x, wy, B.y);
        o = dft_step(o, st, sw);
    }
    if (h == 1 && dv) {
        xs[d] = A;
        xs[32 + d] = B;
    }
    wave_lds_sync();
    if (h == 0 && dv) {
        A = cadd(A, xs[d]);
        B = cadd(B, xs[32 + d]);
    }
    wave_lds_sync();
    if (h == 0 && dv) {
        xs[d] = cadd(c0, cadd(A, B));
        if (d > 0) xs[NSC - d] = cadd(c0, csub(A, B));
    }
    wave_lds_sync();
    return xs[lane < NSC ? lane : 0];
}

// the Gram column -> tap map: kept in LDS (TapsLds) or staged in u[1]
template <typename L>
__device__ __forceinline__ int taps_tap(const L &s, const int *tapl, int j)
{
    if constexpr (L::TAP_MAPS) return s.tap[j];
    else return tapl[j];
}
template <int K0, typename L = SolveLds>
__device__ __forceinline__ void lr_gram_taps(const State *__restrict__ st, L &s, double2 (&A)[RB][RB],
                                             int lane, int p, int q, double ac, double bc, double sl, int tpi)
{
    constexpr int RMAX = NSC - 8 * K0;   // Gram column of the border (row 53)
    constexpr int NB = RB - K0;
    {   // tables: E, p = |x|^2, v = x o conj(rx)
        const double2 xl = s.x[lane], rl = s.rx[lane];
        s.u[1][lane] = cmul(xl, cconj(rl));   // (E is in u[0] since the frame's staging)
        s.rd[lane] = fma(xl.x, xl.x, xl.y * xl.y);
    }
    wave_lds_sync();
    const double2 *E = s.u[0];
    dft_pairs(s.u[1], s.tp.pa, s.tp.pb, lane);
    if (lane >= 1 && lane <= NSC / 2) {
        const double u = s.rd[lane], w = s.rd[NSC - lane];
        s.tp.rp[lane] = make_double2(u + w, u - w);
    }
    wave_lds_sync();
    // Q(d) = sum_k p_k conj(E[k d]), D(d) = sum_k v_k E[k d] on lane d
    // Outputs d and 53 - d share every gather: E[k (53 - d)] = conj(E[k d]), so
    // with A = sum pa_k Re E[k d] and B = i sum pb_k Im E[k d] (over the pairs),
    // D(d) = v_0 + A + B and D(53 - d) = v_0 + A - B; Q(53 - d) = conj(Q(d)).
    // Lane (h, d) = (lane >> 5, lane & 31), d <= 26, sums the pairs k = 1 + 13 h
    // .. 13 + 13 h: 13 steps instead of 26; the halves meet in LDS (blk / z,
    // free until the element build).
    {
        const int h = lane >> 5, d = lane & 31;
        const bool dv = d <= NSC / 2;
        const int dd = dv ? d : 0;
        const int k0 = 1 + (NSC / 4) * h;   // 1 or 14
        const uint32_t st = 16u * (uint32_t)dd, sw = st - 16u * NSC;
        uint32_t o = 16u * (uint32_t)((k0 * dd) % NSC);
        double2 q = make_double2(0.0, 0.0), A = q, B = q;
#pragma unroll 2
        for (int j = 0; j < NSC / 4; ++j) {
            const int k = k0 + j;
            const double2 w = ld_e(E, o), va = s.tp.pa[k], vb = s.tp.pb[k];
            const double2 pp = s.tp.rp[k];   // {p_k + p_{53-k}, p_k - p_{53-k}}
            q.x = fma(pp.x, w.x, q.x);
            q.y = fma(-pp.y, w.y, q.y);
            A.x = fma(va.x, w.x, A.x);
            A.y = fma(va.y, w.x, A.y);
            B.x = fma(-vb.y, w.y, B.x);
            B.y = fma(vb.x, w.y, B.y);
            o = dft_step(o, st, sw);
        }
        if (h == 1 && dv) {
            s.blk[d] = q;
            s.z[d] = A;
            s.z[32 + d] = B;
        }
        wave_lds_sync();
        if (h == 0 && dv) {
            q = cadd(q, s.blk[d]);
            A = cadd(A, s.z[d]);
            B = cadd(B, s.z[32 + d]);
        }
        wave_lds_sync();
        if (h == 0 && dv) {
            const double2 v0 = s.u[1][0];
            const double2 Qp = make_double2(s.rd[0] + q.x, q.y);
            s.blk[d] = cscale(Qp, ac);
            s.z[d] = cadd(v0, cadd(A, B));
            if (d > 0) {
                s.blk[NSC - d] = cscale(cconj(Qp), ac);
                s.z[NSC - d] = cadd(v0, csub(A, B));
            }
        }
    }
    wave_lds_sync();   // every lane's reads of u[1] / the pair tables are done
    // The system is factorised in the scaled form M = S^-1 (a Gamma + b I) S^-1
    // = a T + b S^-2 (T_ij = Q(t_i - t_j)), bordered by S^-1 beta = conj(D(t_j)):
    // its solution is w = S t = the tap vector c of the read-out itself.  A
    // diagonal scaling leaves Cholesky's backward error unchanged (van der
    // Sluis; the dense path's scaled form, s5), and every element is a plain
    // gather of a Q (pre-scaled by a) instead of a product of three factors.
    // Padding columns j in [r, RMAX): pivot b, zero border -> w_j = 0.
    int *tapl = reinterpret_cast<int *>(s.u[1]);   // column j -> its tap (256 B of u[1]) ...
    double *bl = reinterpret_cast<double *>(tapl + 64);   // ... and M's diagonal term b / lambda_j (b past r)
    const int r = st->cov_rank;
    if constexpr (!L::TAP_MAPS) tapl[lane] = tpi;
    bl[lane] = lane < r ? bc / (sl * sl) : bc;
    wave_lds_sync();
#pragma unroll
    for (int m = 0; m < NB; ++m) {
        const int j1 = p + 8 * m;
        const bool v1 = j1 < r;
        const int t1 = taps_tap(s, tapl, j1);
        const double d1 = bl[j1];
#pragma unroll
        for (int n = 0; n <= m; ++n) {
            const int j2 = q + 8 * n;
            const bool v2 = j2 < r;
            const int t2 = taps_tap(s, tapl, j2);
            int dd = t1 - t2;
            dd += dd < 0 ? NSC : 0;
            double2 e;
            if (j1 < RMAX && j2 < RMAX) {
                e = s.blk[dd];
                e = make_double2(v1 && v2 ? e.x : 0.0, v1 && v2 ? e.y : 0.0);
                e.x += j1 == j2 ? d1 : 0.0;
            } else if (j1 == RMAX && j2 < RMAX) {
                e = s.z[t2];
                e = make_double2(v2 ? e.x : 0.0, v2 ? e.y : 0.0);
            } else if (j2 == RMAX && j1 < RMAX) {
                e = cscale(cconj(s.z[t1]), v1 ? ac : 0.0);
            } else {
                e = make_double2(0.0, 0.0);
            }
            A[K0 + m][K0 + n] = e;
        }
        __builtin_amdgcn_sched_barrier(0);   // one block row's gathers in flight at a time
    }
    wave_lds_sync();   // dense_chol reuses u / conv
}

// lr_solve with the tap-domain Gram and read-out (State::cov_taps)
template <int K0, typename L = SolveLds>
__device__ __forceinline__ double2 lr_solve_taps(const State *__restrict__ st, const SolveArgs &a, L &s,
                                                 int64_t base)
{
    const int lane = threadIdx.x;
    const int p = lane >> 3, q = lane & 7;
    const bool act = lane < NSC;
    const double ac = st->acoef, bc = st->bcoef;
    double sl;
    int tpi;
    {   // E, the column -> tap map and s_j in the frame's round trip (E to u[0] now; the map to
        // LDS at the tap stage, or at once with TAP_MAPS, which also keeps tap -> column)
        const double2 t = act ? ld2(a.tx, base + lane) : make_double2(0, 0);
        const double2 r = act ? ld2(a.rx, base + lane) : make_double2(0, 0);
        const bool inx = act && ((st->xmask >> lane) & 1ull);
        const double2 e = act ? ld2(st->dft, lane) : make_double2(0.0, 0.0);
        tpi = st->tap_of[lane];
        sl = st->col_s[lane];
        s.u[0][lane] = e;
        if constexpr (L::TAP_MAPS) {
            s.tap[lane] = (uint8_t)tpi;
            s.col[lane] = (uint8_t)st->col_of[lane];
        }
        s.x[lane] = inx ? t : make_double2(0, 0);
        s.rx[lane] = r;
    }
    wave_lds_sync();
    double2 A[RB][RB];
#pragma unroll
    for (int aa = 0; aa < RB; ++aa)
#pragma unroll
        for (int bb = 0; bb <= aa; ++bb) A[aa][bb] = make_double2(0.0, 0.0);
    lr_gram_taps<K0>(st, s, A, lane, p, q, ac, bc, sl, tpi);
    dense_chol<K0>(A, s, p, q, lane);
    double rq[RB];
#pragma unroll
    for (int bb = 0; bb < RB; ++bb) rq[bb] = s.rd[q + 8 * bb];
    double2 P[RB];
    const bool brow = (p == NSC - 8 * (RB - 1));
#pragma unroll
    for (int bb = 0; bb < RB; ++bb) P[bb] = brow ? cconj(A[RB - 1][bb]) : make_double2(0, 0);
    back_blocks_from<RB - 1, K0>(A, P, rq, s, p, q, lane);
    wave_lds_sync();
    // c_t = s_t t_col(t) = w_col(t) on lane t (w_j = z[8 K0 + j], the scaled system's solution); E back into u[0]
    int col;
    if constexpr (L::TAP_MAPS) {
        const int c8 = s.col[lane];
        col = act && c8 != 0xff ? c8 : -1;
    } else {
        col = act ? st->col_of[lane] : -1;
    }
    {
        const double2 wj = s.z[8 * K0 + (col < 0 ? 0 : col)];
        s.u[1][lane] = col < 0 ? make_double2(0.0, 0.0) : wj;
        s.u[0][lane] = act ? ld2(st->dft, lane) : make_double2(0.0, 0.0);
    }
    wave_lds_sync();
    const double2 *E = s.u[0];
    dft_pairs(s.u[1], s.tp.pa, s.tp.pb, lane);
    wave_lds_sync();
    const double2 xl = s.x[lane];   // re-read: nothing of the frame stays live across the factorisation
    double2 y = lr_dft53_split<false>(E, s.tp.pa, s.tp.pb, s.u[1][0], lane, s.z);   // y_k = sum_t c_t E[k t]
    if (__ballot(act && xl.y != 0.0) != 0) {   // complex symbols: y += U U^H [(x - conj x) o rho] / b
        const double2 rho = csub(s.rx[lane], cscale(cmul(xl, y), ac));   // b Ryy^-1 rx
        s.blk[lane] = act ? make_double2(-2.0 * xl.y * rho.y, 2.0 * xl.y * rho.x) : make_double2(0, 0);
        wave_lds_sync();   // (also: every lane's read-out reads of the pair tables are done)
        dft_pairs(s.blk, s.tp.pa, s.tp.pb, lane);
        wave_lds_sync();
        const double2 w = lr_dft53_split<true>(E, s.tp.pa, s.tp.pb, s.blk[0], lane, s.z);   // w_t = sum_k conj(E[k t]) v_k
        const double ts = st->tap_s[lane];
        s.u[1][lane] = act ? cscale(w, ts * ts / bc) : make_double2(0.0, 0.0);
        wave_lds_sync();
        dft_pairs(s.u[1], s.tp.pa, s.tp.pb, lane);
        wave_lds_sync();
        y = cadd(y, lr_dft53_split<false>(E, s.tp.pa, s.tp.pb, s.u[1][0], lane, s.z));
    }
    return y;
}

// split (MATLAB averaging): one wave per (frame, block) writes H_b to row g
// of a.w; avg_blocks_kernel forms the mean.
// K0 = 0 (r > 45: a Gram system as large as Ryy itself) holds all 28
// register blocks through the product build: 2 waves/SIMD; K0 = 1: 156.
// TAPS: the tap-domain Gram (State::cov_taps), registers as the dense solve's.
constexpr int TAPS_WAVES_K0 = SOLVE_WAVES_PER_SIMD;   // the tap form at K0 = 0 (168 VGPRs, 16 B/lane of scratch at 3 waves/SIMD; 36 before the tap maps moved to LDS)
// K0 >= 2: the LDS holds only rows 8 K0 .. 55 of the panel transposes
// (SolveLdsT<8 K0>: 9.9 KB per wave at K0 = 2 instead of 12.2), so 4 waves per
// SIMD fit a CU's 160 KB where 3.25 did.
constexpr int lr_row0(int k0) { return k0 >= 2 ? 8 * k0 : 0; }
constexpr int LR_TAPS_WAVES = 4;   // the tap form at K0 >= 2 (<= 118 VGPRs)
constexpr int lr_waves(int k0, bool taps)
{
    return taps ? (k0 == 0 ? TAPS_WAVES_K0 : (k0 == 1 ? SOLVE_WAVES_PER_SIMD : LR_TAPS_WAVES))
                : (k0 == 0 ? 2 : (k0 <= 2 ? 3 : LR_WAVES_PER_SIMD));
}
template <int K0, bool TAPS = false>
__global__ __launch_bounds__(64, lr_waves(K0, TAPS)) void mmse_lr_kernel(const State *__restrict__ st, SolveArgs a)
{
    __shared__ std::conditional_t<TAPS && K0 == 0, TapsLds, SolveLdsT<lr_row0(K0)>> s;
    const int64_t g = blockIdx.x;
    const int64_t f = a.split ? g / a.nblk : g;
    const int b = a.split ? (int)(g - f * a.nblk) : 0;
    if (f >= a.n || (a.skip && a.skip[g])) return;   // skip: H already written (constant-modulus path)
    const int64_t base = f * a.fs + (int64_t)(a.blk + b) * a.bs;
    double2 h;
    if constexpr (TAPS) h = lr_solve_taps<K0>(st, a, s, base);
    else h = lr_solve<K0>(st, a, s, base);
    if (threadIdx.x < NSC) st2(a.w, g * a.ws + threadIdx.x, h);
}

// ---------------------------------------------------------------------
// The same low-rank MMSE for ranks 1..LRL_RMAX, ONE (frame, block) PER LANE.
// At rank <= 8 the Gram system is tiny (36 complex entries), so a wave per
// frame spends its time on latency: the embedded 8 x 8-block factorisation
// runs whole pivot chains for a handful of live rows, and 12 KB of LDS per
// wave caps a CU at 13 waves (0.147 ms per 65,536 frames at rank 4, 0.268 at
// rank 8, against ~0.035 ms for the 167 MB the frames and H move).  Here the
// shared factors are wave-uniform and every lane owns its frame outright:
//   pass 1, k = 0..52:  Gamma += |x_k|^2 P_k   (P_k[i][j] = conj(U_ki) U_kj,
//                       State::Pk, scalar loads), beta += conj(U_k) conj(x_k) rx_k
//   (a Gamma + b I) t = beta: Cholesky + two triangular solves in registers
//   complex x only (wave-uniform branch): s = t + U^H [(x - conj x) o
//                       (rx - a x o (U t))] / b, one more pass over k
//   pass 2, k = 0..52:  H_k = U_k s, stored straight from the lane.
// Same algebra as mmse_lr_kernel (G = X U, border Gamma^H rx), summed in
// another order: the two agree to ~1e-15 (tests/test_cov_lowrank_gpu.py).
// No LDS, no cross-lane traffic; the frame's loads and stores are 16 B per
// lane at the frame stride, consecutive k filling each 64-B sector in turn.
// ---------------------------------------------------------------------
// Memory, two forms (launch_mmse_lr picks by batch size):
//  - direct (STAGED = false): each lane loads its frame's 16 B per subcarrier
//    and stores H the same way, 4 subcarriers (one 64-B sector) per unrolled
//    step.  Best while the grid is small: 0.052 ms at rank 4 for 65,536
//    frames.  But every instruction touches 64 sectors, and from 131,072
//    frames on the resident waves keep enough partly-read sectors live to
//    thrash the caches: 0.143 ms at 131,072, 1.28 ms at 1,048,576 (2.1 TB/s).
//  - staged (STAGED = true): the wave moves its 64 frames through LDS in
//    chunks of 4 subcarriers, coalesced (16 frames x 64 B per instruction),
//    each chunk's loads issued one chunk ahead into registers; every lane then
//    reads its own frame's 4 values from LDS (row stride 5 complex:
//    conflict-free), and H goes out the same way in reverse.  0.110 ms at
//    131,072 frames, 0.95 ms at 1,048,576, but 0.061 ms at 65,536.  H leaves
//    in chunks of 8 subcarriers (8 frames x 128 B per store, 7 stores per
//    frame instead of 14 of 64 B): rank 8 0.055 -> 0.046 ms at 65,536 frames,
//    2.7-4% at 1,048,576, bit-identical (profiles/r04_ab_lowrank_store8.txt).
constexpr int LR_LANE_UNROLL = 4;   // direct form without the look-ahead: subcarriers per step up to rank 4
constexpr int LR_LDS_P = 0x110;     // direct form: P_k and U staged in LDS per workgroup instead of scalar loads, for the
                                    // ranks whose bit is set: 4 and 8 (measured per rank, profiles/r03_ab_lowrank_ldsp.txt)
constexpr int LRL_KC = 4;                         // subcarriers per chunk
constexpr int LRL_NCH = (NSC + LRL_KC - 1) / LRL_KC;   // 14 chunks (k = 52..55: only 52 is live)
constexpr int LRL_LS = 5;                         // LDS row stride (complex) per frame
struct LrLaneLds {
    double2 x[64 * LRL_LS];
    double2 r[64 * LRL_LS];
};
// the wave's chunk c of tx / rx as 4 x 16 B per lane: element e = lane + 64 m
// is frame e >> 2 of the wave, subcarrier 4 c + (e & 3)
struct LrChunk {
    double2 x[4], r[4];
};
__device__ __forceinline__ void lrl_load(LrChunk &q, const SolveArgs &a, const int64_t (&eb)[4], uint32_t live,
                                         int c, int lane)
{
    const int k = LRL_KC * c + (lane & 3);
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const bool ok = ((live >> m) & 1u) && k < NSC;
        // plain loads: the 64-B pieces straddle sectors (frames 848 B apart), and the
        // next chunk's load finds the shared sector in L2 (nontemporal: 0.89 -> 1.63 ms
        // at 1,048,576 frames, profiles/r04_ab_lowrank_nt.txt)
        q.x[m] = ok ? ld2(a.tx, eb[m] + k) : make_double2(0.0, 0.0);
        q.r[m] = ok ? ld2(a.rx, eb[m] + k) : make_double2(0.0, 0.0);
    }
}
__device__ __forceinline__ void lrl_stage(LrLaneLds &s, const LrChunk &q, int lane)
{
    asm volatile("" ::: "memory");   // after the previous chunk's reads (LDS runs a wave's ops in order)
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const int fl = (lane >> 2) + 16 * m;
        s.x[fl * LRL_LS + (lane & 3)] = q.x[m];
        s.r[fl * LRL_LS + (lane & 3)] = q.r[m];
    }
    asm volatile("" ::: "memory");
}
// pass-1 / correction-pass sweep over k: f(k, x_k, rx_k) in order k = 0..52
template <bool STAGED, int UN, typename Fn>
__device__ __forceinline__ void lrl_sweep(LrLaneLds *sp, const SolveArgs &a, const int64_t (&eb)[4], uint32_t live,
                                          int64_t base, bool own, int lane, Fn fn)
{
    if constexpr (STAGED) {
        LrChunk q;
        lrl_load(q, a, eb, live, 0, lane);
#pragma unroll 1
        for (int c = 0; c < LRL_NCH; ++c) {
            lrl_stage(*sp, q, lane);
            if (c + 1 < LRL_NCH) lrl_load(q, a, eb, live, c + 1, lane);   // one chunk ahead
#pragma unroll
            for (int kk = 0; kk < LRL_KC; ++kk) {
                const int k = LRL_KC * c + kk;
                if (kk > 0 && k >= NSC) break;   // (uniform) the last chunk holds k = 52 only
                fn(k, sp->x[lane * LRL_LS + kk], sp->r[lane * LRL_LS + kk]);
            }
        }
    } else {
#pragma unroll UN
        for (int k = 0; k < NSC; ++k)
            fn(k, own ? ld2(a.tx, base + k) : make_double2(0.0, 0.0), own ? ld2(a.rx, base + k) : make_double2(0.0, 0.0));
    }
}
// Pl / Ul (LR_LDS_P, direct form): the workgroup's LDS copies of P_k
// (R (R + 1) / 2 entries per k) and U (R per k); else State::Pk / State::U
// TQ (State::taps_contig, staged form with LDS tables): Pl holds E[k s mod 53]
// (R per k) instead of P_k, and pass 1 accumulates the Toeplitz Gram's R
// values Q(s) = sum_k |x_k|^2 conj(E[k s]) (2 FMAs each per subcarrier) instead
// of its R (R + 1) / 2 products; Gamma_ij = s_i s_j Q(i - j) afterwards.
template <int R, bool STAGED, bool LP = false, bool TQ = false>
__device__ __forceinline__ void lr_lane_body(const State *__restrict__ st, const SolveArgs &a, LrLaneLds *sp,
                                             int fpw, const double2 *Pl = nullptr, const double2 *Ul = nullptr)
{
    static_assert(!TQ || LP, "the Toeplitz pass reads its E table from LDS");
    constexpr int NO = R * (R - 1) / 2;   // strictly-lower Gram entries
    const int lane = threadIdx.x & 63;
    const int64_t units = a.split ? a.n * a.nblk : a.n;
    // the wave's first (frame, block) unit; the direct form may run fpw < 64
    // units per wave (lanes past fpw idle) to put more waves on a small batch
    const int64_t g0 = ((int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * fpw;
    const int64_t g = g0 + lane;
    const bool own = lane < fpw && g < units;
    if (!STAGED && !own) return;   // (a staging wave moves all 64 lanes' data)
    auto ubase = [&](int64_t u) {   // (frame, block) unit -> element offset of its block
        const int64_t f = a.split ? u / a.nblk : u;
        const int b = a.split ? (int)(u - f * a.nblk) : 0;
        return f * a.fs + (int64_t)(a.blk + b) * a.bs;
    };
    const int64_t base = own ? ubase(g) : 0;
    int64_t eb[4];   // STAGED: the unit element lane + 64 m stages
    uint32_t live = 0;
#pragma unroll
    for (int m = 0; m < 4; ++m) {
        const int64_t u = g0 + (lane >> 2) + 16 * m;
        live |= ((lane >> 2) + 16 * m < fpw && u < units ? 1u : 0u) << m;
        eb[m] = STAGED && u < units ? ubase(u) : 0;
    }
    const double ac = st->acoef, bc = st->bcoef;
    const uint64_t xm = st->xmask;
    constexpr int NPR = R * (R + 1) / 2;
    const double2 *__restrict__ P = LP ? Pl : reinterpret_cast<const double2 *>(st->Pk);
    const double2 *__restrict__ U = LP ? Ul : reinterpret_cast<const double2 *>(st->U);
    constexpr int pld = LP ? NPR : LRL_NP, uld = LP ? R : CLD;
    double gd[R];        // Gamma_ii (real)
    double2 go[NO > 0 ? NO : 1];   // Gamma_ij, i > j, at i (i - 1) / 2 + j
    double2 bt[R];       // beta = G^H rx
#pragma unroll
    for (int i = 0; i < R; ++i) {
        gd[i] = 0.0;
        bt[i] = make_double2(0.0, 0.0);
    }
#pragma unroll
    for (int e = 0; e < NO; ++e) go[e] = make_double2(0.0, 0.0);
    bool cplx = false;
    constexpr int UN = R <= 4 ? LR_LANE_UNROLL : 1;   // ranks 5..8: the Gram registers leave no room
    if constexpr (TQ) {
        double q0 = 0.0;                      // Q(0) (real)
        double2 qs[R > 1 ? R - 1 : 1];        // Q(1..R-1)
#pragma unroll
        for (int e = 0; e < R - 1; ++e) qs[e] = make_double2(0.0, 0.0);
        lrl_sweep<STAGED, UN>(sp, a, eb, live, base, own, lane, [&](int k, double2 x, double2 r) {
            if (!((xm >> k) & 1ull)) x = make_double2(0.0, 0.0);
            cplx |= x.y != 0.0;
            const double w = fma(x.x, x.x, x.y * x.y);
            const double2 v = make_double2(fma(x.x, r.x, x.y * r.y), fma(x.x, r.y, -x.y * r.x));   // conj(x) rx
            const double2 *Ek = P + k * R;   // E[k s mod 53], s < R
#pragma unroll
            for (int i = 0; i < R; ++i) {
                const double2 u = U[k * uld + i];   // beta_i += conj(u) v
                bt[i].x = fma(u.x, v.x, fma(u.y, v.y, bt[i].x));
                bt[i].y = fma(u.x, v.y, fma(-u.y, v.x, bt[i].y));
            }
            q0 += w;
#pragma unroll
            for (int e = 1; e < R; ++e) {   // += w conj(E[k e])
                const double2 ee = Ek[e];
                qs[e - 1].x = fma(w, ee.x, qs[e - 1].x);
                qs[e - 1].y = fma(-w, ee.y, qs[e - 1].y);
            }
        });
        // Gamma_ij = s_i s_j Q(i - j): s wave-uniform (scalar loads)
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const double si = st->col_s[i];
            gd[i] = si * si * q0;
#pragma unroll
            for (int j = 0; j < i; ++j) go[i * (i - 1) / 2 + j] = cscale(qs[i - j - 1], si * st->col_s[j]);
        }
    } else {
    lrl_sweep<STAGED, UN>(sp, a, eb, live, base, own, lane, [&](int k, double2 x, double2 r) {
        if (!((xm >> k) & 1ull)) x = make_double2(0.0, 0.0);
        cplx |= x.y != 0.0;
        const double w = fma(x.x, x.x, x.y * x.y);
        const double2 v = make_double2(fma(x.x, r.x, x.y * r.y), fma(x.x, r.y, -x.y * r.x));   // conj(x) rx
        const double2 *Pk = P + k * pld;
#pragma unroll
        for (int i = 0; i < R; ++i) {
            const double2 u = U[k * uld + i];   // beta_i += conj(u) v
            bt[i].x = fma(u.x, v.x, fma(u.y, v.y, bt[i].x));
            bt[i].y = fma(u.x, v.y, fma(-u.y, v.x, bt[i].y));
            gd[i] = fma(w, Pk[i * (i + 1) / 2 + i].x, gd[i]);
#pragma unroll
            for (int j = 0; j < i; ++j) {
                const double2 pe = Pk[i * (i + 1) / 2 + j];
                double2 &o = go[i * (i - 1) / 2 + j];
                o.x = fma(w, pe.x, o.x);
                o.y = fma(w, pe.y, o.y);
            }
        }
    });
    }
    // A = a Gamma + b I = L L^H (lower L in place: ld = 1 / L_ii, lo = L_ij)
    double ld[R];
    double2 lo[NO > 0 ? NO : 1];
#pragma unroll
    for (int i = 0; i < R; ++i) {
#pragma unroll
        for (int j = 0; j < i; ++j) {
            double2 acc = cscale(go[i * (i - 1) / 2 + j], ac);
#pragma unroll
            for (int m = 0; m < j; ++m) {   // acc -= L_im conj(L_jm)
                const double2 x = lo[i * (i - 1) / 2 + m], y = lo[j * (j - 1) / 2 + m];
                acc.x = fma(-x.x, y.x, fma(-x.y, y.y, acc.x));
                acc.y = fma(-x.y, y.x, fma(x.x, y.y, acc.y));
            }
            lo[i * (i - 1) / 2 + j] = cscale(acc, ld[j]);
        }
        double d = fma(ac, gd[i], bc);
#pragma unroll
        for (int m = 0; m < i; ++m) {
            const double2 x = lo[i * (i - 1) / 2 + m];
            d = fma(-x.x, x.x, fma(-x.y, x.y, d));
        }
        ld[i] = 1.0 / sqrt(d);
    }
    // t = L^-H L^-1 beta
    double2 t[R];
#pragma unroll
    for (int i = 0; i < R; ++i) {
        double2 acc = bt[i];
#pragma unroll
        for (int m = 0; m < i; ++m) acc = csub(acc, cmul(lo[i * (i - 1) / 2 + m], t[m]));
        t[i] = cscale(acc, ld[i]);
    }
#pragma unroll
    for (int i = R - 1; i >= 0; --i) {
        double2 acc = t[i];
#pragma unroll
        for (int m = i + 1; m < R; ++m) acc = csub(acc, cmul(cconj(lo[m * (m - 1) / 2 + i]), t[m]));
        t[i] = cscale(acc, ld[i]);
    }
    if (__ballot(cplx) != 0) {   // complex symbols: s = t + U^H [(x - conj x) o (rx - a x o (U t))] / b
        double2 cc[R];
#pragma unroll
        for (int i = 0; i < R; ++i) cc[i] = make_double2(0.0, 0.0);
        lrl_sweep<STAGED, 2>(sp, a, eb, live, base, own, lane, [&](int k, double2 x, double2 r) {
            if (!((xm >> k) & 1ull)) x = make_double2(0.0, 0.0);
            // the products accumulate as FMA chains (4 per complex term, where
            // cadd(y, cmul(u, t)) rounds the product first: 6)
            double2 y = make_double2(0.0, 0.0);
#pragma unroll
            for (int j = 0; j < R; ++j) {
                const double2 u = U[k * uld + j];
                y.x = fma(u.x, t[j].x, fma(-u.y, t[j].y, y.x));
                y.y = fma(u.x, t[j].y, fma(u.y, t[j].x, y.y));
            }
            const double2 rho = csub(r, cscale(cmul(x, y), ac));
            const double2 v = make_double2(-2.0 * x.y * rho.y, 2.0 * x.y * rho.x);
#pragma unroll
            for (int j = 0; j < R; ++j) {   // cc_j += conj(u) v
                const double2 u = U[k * uld + j];
                cc[j].x = fma(u.x, v.x, fma(u.y, v.y, cc[j].x));
                cc[j].y = fma(u.x, v.y, fma(-u.y, v.x, cc[j].y));
            }
        });
        const double rb = 1.0 / bc;
#pragma unroll
        for (int i = 0; i < R; ++i) t[i] = cadd(t[i], cscale(cc[i], rb));
    }
    // H_k = U_k s
    auto hk = [&](int k) {
        double2 y = make_double2(0.0, 0.0);
#pragma unroll
        for (int j = 0; j < R; ++j) {
            const double2 u = U[k * uld + j];
            y.x = fma(u.x, t[j].x, fma(-u.y, t[j].y, y.x));
            y.y = fma(u.x, t[j].y, fma(u.y, t[j].x, y.y));
        }
        return y;
    };
    if constexpr (STAGED) {   // each lane its frame's 8 subcarriers of a chunk into LDS (x and r as one
                              // area), then 8 frames x 128 B per store: a frame's H in 7 stores, not 14
        constexpr int SC = 8, SS = 9;   // subcarriers per store chunk, LDS row stride (complex) per frame
        static_assert(sizeof(LrLaneLds) >= 64 * SS * sizeof(double2), "store staging fits the chunk buffers");
        double2 *so = sp->x;
        int64_t ob[8];
        uint32_t live8 = 0;
#pragma unroll
        for (int m = 0; m < 8; ++m) {
            const int64_t u = g0 + (lane >> 3) + 8 * m;
            ob[m] = u * a.ws;
            live8 |= (u < units ? 1u : 0u) << m;
        }
#pragma unroll 1
        for (int c = 0; c < (NSC + SC - 1) / SC; ++c) {
            asm volatile("" ::: "memory");
#pragma unroll
            for (int kk = 0; kk < SC; ++kk) {
                const int k = SC * c + kk;
                if (kk > 0 && k >= NSC) break;
                so[lane * SS + kk] = hk(k);
            }
            asm volatile("" ::: "memory");
            const int k = SC * c + (lane & 7);
#pragma unroll
            for (int m = 0; m < 8; ++m) {
                const double2 y = so[((lane >> 3) + 8 * m) * SS + (lane & 7)];
                if (((live8 >> m) & 1u) && k < NSC) st2(a.w, ob[m] + k, y);
            }
        }
    } else {
        double *W = a.w + 2 * g * a.ws;
#pragma unroll 4
        for (int k = 0; k < NSC; ++k) st2(W, k, hk(k));
    }
}
template <int R>
__global__ __launch_bounds__(256) void mmse_lr_lane_kernel(const State *__restrict__ st, SolveArgs a, int fpw)
{
    if constexpr (((LR_LDS_P >> R) & 1) != 0) {
    // P_k and U through LDS: their scalar loads each wait a round trip per k
    // (18 s_load_dwordx16 per k at rank 8, and rank 8's 30 KB of P_k does not
    // stay in the scalar cache), fully exposed at one wave per SIMD.  Per rank
    // at 65,536 frames: rank 8 98.0 -> 68.7 us, rank 4 54.9 -> 50.3 us, but
    // ranks 3, 5, 6, 7 slower (52.6 -> 59.0, 62.6 -> 93.7, 65.4 -> 67.1,
    // 74.8 -> 84.7: the LDS reads cost VGPRs and the compiler's schedule
    // changes with them), rank 1, 2 equal; bit-identical everywhere
    constexpr int NPR = R * (R + 1) / 2;
    __shared__ double2 sP[NSC * NPR], sU[NSC * R];
    const double2 *Pg = reinterpret_cast<const double2 *>(st->Pk);
    const double2 *Ug = reinterpret_cast<const double2 *>(st->U);
    for (int e = threadIdx.x; e < NSC * NPR; e += blockDim.x) sP[e] = Pg[(e / NPR) * LRL_NP + e % NPR];
    for (int e = threadIdx.x; e < NSC * R; e += blockDim.x) sU[e] = Ug[(e / R) * CLD + e % R];
    __syncthreads();
    lr_lane_body<R, false, true>(st, a, nullptr, fpw, sP, sU);
    } else {
        lr_lane_body<R, false>(st, a, nullptr, fpw);
    }
}
// staged form: 4-wave workgroups sharing one LDS copy of P_k and U, for the ranks whose bit is set: every rank
// (1,048,576 frames, rank 8 1476 -> 951 us, 7 1343 -> 875, 6 1189 -> 845, 5 894 -> 840, 2 952 -> 934, 4 equal;
// profiles/r03_ab_lowrank_ldsp.txt)
constexpr int LR_STAGED_LDS_P = 0x1fe;
// 4-wave workgroups per CU asked of the register allocator, ranks >= 7, batches past one wave per SIMD.
// 1,048,576 frames: rank 7 898 -> 858 us, rank 8 955 -> 896 (2 waves/SIMD instead of 1; rank 8 spills 52 B);
// at 65,536 frames (one wave per SIMD anyway) rank 8 63.3 -> 67.5, so MW = 1 there
constexpr int LR_STAGED_MINWG = 2;
constexpr int lr_staged_threads(int r) { return ((LR_STAGED_LDS_P >> r) & 1) ? 256 : 64; }
template <int R, int MW = 1, bool TQ = false>
__global__ __launch_bounds__(lr_staged_threads(R), MW) void mmse_lr_lane_staged_kernel(const State *__restrict__ st, SolveArgs a)
{
    if constexpr (lr_staged_threads(R) == 256) {
        constexpr int NPR = TQ ? R : R * (R + 1) / 2;   // TQ: E[k s mod 53], s < R
        __shared__ double2 sP[NSC * NPR], sU[NSC * R];
        __shared__ LrLaneLds s[4];
        const double2 *Pg = reinterpret_cast<const double2 *>(st->Pk);
        const double2 *Ug = reinterpret_cast<const double2 *>(st->U);
        {   // P_k (TQ: E[k s]) and U: every load issued before the first LDS store
            constexpr int NP = NSC * NPR, NU = NSC * R;
            constexpr int IP = (NP + 255) / 256, IU = (NU + 255) / 256;
            double2 vp[IP], vu[IU];
#pragma unroll
            for (int it = 0; it < IP; ++it) {
                const int e = min((int)threadIdx.x + 256 * it, NP - 1);
                if constexpr (TQ) vp[it] = ld2(st->dft, ((e / NPR) * (e % NPR)) % NSC);
                else vp[it] = Pg[(e / NPR) * LRL_NP + e % NPR];
            }
#pragma unroll
            for (int it = 0; it < IU; ++it) {
                const int e = min((int)threadIdx.x + 256 * it, NU - 1);
                vu[it] = Ug[(e / R) * CLD + e % R];
            }
            // stores unguarded: a thread past the end rewrites the last element with
            // the value it loaded from there (a guard lets the compiler sink the
            // loads into it, one round trip each)
#pragma unroll
            for (int it = 0; it < IP; ++it) sP[min((int)threadIdx.x + 256 * it, NP - 1)] = vp[it];
#pragma unroll
            for (int it = 0; it < IU; ++it) sU[min((int)threadIdx.x + 256 * it, NU - 1)] = vu[it];
        }
        __syncthreads();
        lr_lane_body<R, true, true, TQ>(st, a, &s[threadIdx.x >> 6], 64, sP, sU);
    } else {
        static_assert(!TQ, "the Toeplitz form runs in the 4-wave LDS-table build");
        __shared__ LrLaneLds s;
        lr_lane_body<R, true>(st, a, &s, 64);
    }
}

// ---------------------------------------------------------------------
// Ranks 9..16: 16 LANES PER (frame, block), 4 per wave (mmse_lr_quad_kernel).
// A rank-16 Gram system no longer fits one lane's registers (136 complex
// entries), and a wave per frame spends most of its time on the 53-row
// machinery around a 16-row system (0.447 ms per 65,536 frames at rank 16).
// Here lane i of a 16-lane DPP row holds row i of the system:
//   pass 1, k = 0..52:  Gamma[i][:] += w_k conj(U_ki) U_k:   (U_k: scalar loads,
//                       conj(U_ki): the lane's own), beta_i += conj(U_ki) conj(x_k) rx_k
//   Cholesky on the rows: pivot c's scale and column by row_newbcast:c inside
//                       the 16-lane row (DPP, no LDS), the trailing rows updated
//                       by each lane for its own row
//   z = L^-1 beta column by column, z_c as the DPP64 row_newbcast operand of
//                       the FMAs (round 6); t = L^-H z by 16-lane DPP sums
//                       (column c of L is spread over the rows, one per lane)
//   complex x (a wave-uniform branch): the correction term from the lane's 4
//                       subcarriers k = i, i + 16, ..., summed over the row
//   H_k = U_k s for the lane's 4 subcarriers: 16 lanes store 256 B of one frame.
// Same algebra as mmse_lr_kernel, summed in another order (~1e-15).
// ---------------------------------------------------------------------
// FD (round 6): L[j][C] as the DPP64 row_newbcast operand of the update FMAs
// (cmsub_dpp: 4 VALU per update instead of 2 movs + 4 FMAs), bit-identical
template <int R, int C, bool FD = true>
__device__ __forceinline__ void lrq_chol(double2 (&Ar)[R], double &ldi, int i)
{
    if constexpr (C < R) {
        const double d = row_bcast<C>(Ar[C]).x;   // pivot (C, C), from lane C of the row
        const double rs = rsq_nr(d);
        Ar[C] = cscale(Ar[C], rs);                 // L[i][C] (for i >= C)
        ldi = i == C ? rs : ldi;                   // 1 / L_ii
        if constexpr (FD) dpp_ready(Ar[C]);
#pragma unroll
        for (int j = C + 1; j < R; ++j) {          // A[i][j] -= L[i][C] conj(L[j][C])
            if constexpr (FD) {
                cmsub_dpp_n(j, Ar[j], Ar[C], Ar[C]);
            } else {
                const double2 lj = row_bcast_n(Ar[C], j);
                cmsub_conj(Ar[j], Ar[C], lj);
            }
        }
        lrq_chol<R, C + 1, FD>(Ar, ldi, i);
    }
}

// One 16-lane unit's LDS in mmse_lr_quad_kernel<R, true> (1,344 B, so that 4
// workgroups fit a CU: the kernel needs <= 128 VGPRs since round 6): the frame's
// v = conj(x) o rx and p = |x|^2, turned in place into the pair tables
// (V[k] = v_k + v_{53-k}, V[53-k] = v_k - v_{53-k}, RP[k] = {p_k + p_{53-k},
// p_k - p_{53-k}} over W), then Q(0..15) over V.  The unit pitch (84 slots of
// 16 B, 4 mod 16) puts two units' same-index reads in one ds_read_b128 lane
// group on different banks.
struct LrqTabs {
    double2 V[56];
    double W[56];
};
static_assert(sizeof(LrqTabs) / 16 % 16 != 0, "unit pitch not 0 mod 16 slots");

// (pass 1's U_k from an LDS copy per workgroup instead of scalar loads: slower,
// rank 16 237 -> 271 us at 65,536 frames, 3.82 -> 4.39 ms at 1M; retired in
// round 4, profiles/r03_ab_lowrank_ldsp.txt: U, 13.6 KB at rank 16, stays in
// the scalar cache, and 3 waves/SIMD hide its latency)
// TQ (State::taps_contig: a power-delay profile whose kept taps are 0..R-1,
// column j = tap j): Gamma = S Q S with Q(i - j) = sum_k p_k conj(E[k (i - j)])
// Toeplitz, so pass 1 accumulates ONE Gram value per lane, Q(i) (2 FMAs per
// subcarrier, E[k i mod 53] from an LDS copy of State::dft by the exact index
// recurrence), instead of its row of R products (4R FMAs): the row's values
// meet in LDS and lane i reads Q(|i - j|) (conjugated for j > i).
template <int R, bool TQ = false, bool FD = true>
__global__ __launch_bounds__(256) void mmse_lr_quad_kernel(const State *__restrict__ st, SolveArgs a)
{
    const int i = threadIdx.x & 15;   // the row of the R x R system this lane holds
    const int64_t units = a.split ? a.n * a.nblk : a.n;
    const int64_t g = ((int64_t)blockIdx.x * 256 + threadIdx.x) >> 4;   // (frame, block) unit of the row
    const double2 *__restrict__ U1 = reinterpret_cast<const double2 *>(st->U);   // wave-uniform: scalar loads
    constexpr int uld = CLD;
    __shared__ double2 sE[TQ ? 64 : 1];
    __shared__ LrqTabs sU[TQ ? 16 : 1];   // the workgroup's 16 units
    const int rw = (threadIdx.x >> 4) & 15;
    if constexpr (TQ) {
        if (threadIdx.x < 64) sE[threadIdx.x] = ld2(st->dft, threadIdx.x);
        __syncthreads();
    }
    if (g >= units || (a.skip && a.skip[g])) return;   // whole 16-lane rows (skip: the constant-modulus path wrote H)
    const int64_t f = a.split ? g / a.nblk : g;
    const int b = a.split ? (int)(g - f * a.nblk) : 0;
    const int64_t base = f * a.fs + (int64_t)(a.blk + b) * a.bs;
    const double ac = st->acoef, bc = st->bcoef;
    const uint64_t xm = st->xmask;
    const double2 *__restrict__ UT = reinterpret_cast<const double2 *>(st->UT);
    const bool row = i < R;
    double2 Ar[R];   // row i of Gamma, then of a Gamma + b I, then of L
#pragma unroll
    for (int j = 0; j < R; ++j) Ar[j] = make_double2(0.0, 0.0);
    double2 bt = make_double2(0.0, 0.0);
    bool cplx = false;
    if constexpr (TQ) {
        // the row's frame through LDS: lane i loads subcarriers i, i + 16, ... (256 B
        // per row and instruction), then every lane sweeps k from broadcast reads
        LrqTabs &T = sU[rw];
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const int k = i + 16 * m;
            if (k < NSC) {
                double2 x = ld2(a.tx, base + k);
                const double2 r = ld2(a.rx, base + k);
                if (!((xm >> k) & 1ull)) x = make_double2(0.0, 0.0);
                cplx |= x.y != 0.0;
                T.W[k] = fma(x.x, x.x, x.y * x.y);
                T.V[k] = make_double2(fma(x.x, r.x, x.y * r.y), fma(x.x, r.y, -x.y * r.x));   // conj(x) rx
            }
        }
        wave_lds_sync();   // the row's 16 lanes are one wave's
        // pair tables over (k, 53 - k), k = 1..26 (round 6, as mmse_lr_quad2_kernel):
        // one gather and half the FMAs per pair; in place, so every read first
        double2 *RP = reinterpret_cast<double2 *>(T.W);   // RP[k] over W[2k], W[2k + 1], k >= 1
        double2 u[2], w[2];
        double pu[2], pw[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int kp = i + 1 + 16 * h, kc = kp <= NSC / 2 ? kp : 1;
            u[h] = T.V[kc];
            w[h] = T.V[NSC - kc];
            pu[h] = T.W[kc];
            pw[h] = T.W[NSC - kc];
        }
        wave_lds_sync();
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int kp = i + 1 + 16 * h;
            if (kp <= NSC / 2) {
                T.V[kp] = cadd(u[h], w[h]);
                T.V[NSC - kp] = csub(u[h], w[h]);
                RP[kp] = make_double2(pu[h] + pw[h], pu[h] - pw[h]);
            }
        }
        wave_lds_sync();
        // Q(i) = sum_k p_k conj(E[k i]), beta_i = s_i sum_k v_k conj(E[k i]) (U[k][i] = s_i E[k i])
        double2 q = make_double2(T.W[0], 0.0), bq = T.V[0];   // the k = 0 terms
        const uint32_t qs = 16u * (uint32_t)i, qw = qs - 16u * NSC;
        uint32_t qo = qs;   // 16 (k i mod 53), k = 1
#pragma unroll 2
        for (int kp = 1; kp <= NSC / 2; ++kp) {
            const double2 e = ld_e(sE, qo), pa = T.V[kp], pb = T.V[NSC - kp], pp = RP[kp];
            q.x = fma(pp.x, e.x, q.x);
            q.y = fma(-pp.y, e.y, q.y);
            bq.x = fma(pa.x, e.x, fma(pb.y, e.y, bq.x));
            bq.y = fma(pa.y, e.x, fma(-pb.x, e.y, bq.y));
            qo = dft_step(qo, qs, qw);
        }
        const double si = row ? st->col_s[i] : 0.0;
        bt = cscale(bq, si);
        wave_lds_sync();   // every lane's table reads are done: Q(i) over V
        T.V[i] = q;
        wave_lds_sync();
#pragma unroll
        for (int j = 0; j < R; ++j) {   // a s_i s_j Q(i - j) + b [i == j]; rows past R: the identity (never read)
            const double2 qd = j <= i ? T.V[(i - j) & 15] : cconj(T.V[(j - i) & 15]);
            Ar[j] = cscale(qd, ac * si * st->col_s[j]);
            Ar[j].x += (i == j || (!row && j == 0)) ? bc : 0.0;
        }
    } else {
#pragma unroll 1
        for (int k = 0; k < NSC; ++k) {
            double2 x = ld2(a.tx, base + k);   // the same 16 B in the row's 16 lanes
            const double2 r = ld2(a.rx, base + k);
            if (!((xm >> k) & 1ull)) x = make_double2(0.0, 0.0);
            cplx |= x.y != 0.0;
            const double w = fma(x.x, x.x, x.y * x.y);
            const double2 v = make_double2(fma(x.x, r.x, x.y * r.y), fma(x.x, r.y, -x.y * r.x));   // conj(x) rx
            const double2 ui = row ? U1[k * uld + i] : make_double2(0.0, 0.0);
            bt.x = fma(ui.x, v.x, fma(ui.y, v.y, bt.x));   // += conj(u_i) v
            bt.y = fma(ui.x, v.y, fma(-ui.y, v.x, bt.y));
            const double2 wi = make_double2(w * ui.x, -w * ui.y);   // w conj(u_i)
#pragma unroll
            for (int j = 0; j < R; ++j) {
                const double2 uj = U1[k * uld + j];   // wave-uniform: scalar loads (or an LDS broadcast)
                Ar[j].x = fma(wi.x, uj.x, fma(-wi.y, uj.y, Ar[j].x));
                Ar[j].y = fma(wi.x, uj.y, fma(wi.y, uj.x, Ar[j].y));
            }
        }
#pragma unroll
        for (int j = 0; j < R; ++j) {   // a Gamma + b I; rows past R: the identity (never read)
            Ar[j] = cscale(Ar[j], ac);
            Ar[j].x += (i == j || (!row && j == 0)) ? bc : 0.0;
        }
    }
    double ldi = 1.0;
    lrq_chol<R, 0, FD>(Ar, ldi, i);
    // z = L^-1 beta: lane i keeps y_i = beta_i - sum_{c < i} L[i][c] z_c, and
    // z_c = y_c / L_cc reaches the FMAs from lane c as their DPP64 row_newbcast
    // operand (conj(z_c) in w: cmsub_dpp subtracts l conj(R)).  L's entries on
    // and above the diagonal are zeroed first, so that no lane needs a select
    // here or in the back-substitution (round 6: 2 muls and 4 DPP FMAs per
    // column where a broadcast, a product and selects took ~20 VALU).
#pragma unroll
    for (int c = 0; c < R; ++c) keep_where_mask(rows16_upto(c), true, Ar[c], make_double2(0.0, 0.0));
    double2 yv = bt;
#pragma unroll
    for (int c = 0; c < R; ++c) {
        double2 w = make_double2(yv.x * ldi, -(yv.y * ldi));
        dpp_ready(w);
        cmsub_dpp_n(c, yv, Ar[c], w);   // y_i -= L[i][c] z_c
    }
    const double2 z = cscale(yv, ldi);
    // t = L^-H z: t_c = (z_c - sum_{m > c} conj(L[m][c]) t_m) / L_cc, the sum
    // over the row's lanes (column c of L is spread over them; lanes m <= c
    // hold a zero or a t_m still zero).  (Round 6 A/B: L's rows through LDS so
    // that lane c reads its column, t_m as the DPP operand, measured 3-5%
    // slower at ranks 12..20 and 12% at 24, profiles/r06_ab_lowrank_solves.txt.)
    double2 t = make_double2(0.0, 0.0);
#pragma unroll
    for (int c = R - 1; c >= 0; --c) {
        const double2 sum = row16_sum(cmul(cconj(Ar[c]), t));
        if (i == c) t = cscale(csub(z, sum), ldi);
    }
    double *W = a.w + 2 * g * a.ws;
    if constexpr (TQ) {
        if (__ballot(cplx) != 0) {   // complex symbols, in the tap domain (round 6): see lrq_cplx_taps
            LrqTabs &T = sU[rw];
            const double si = row ? st->col_s[i] : 0.0;
            double2 c = cscale(t, si), cb = c;   // (cb: rows i + 16, none here)
            lrq_cplx_taps<R>(xm, a.tx, a.rx, base, sE, T.V, c, cb, i, ac, bc);
            t = cadd(t, cscale(c, si));
        }
    } else if (__ballot(cplx) != 0) {   // complex symbols: s = t + U^H [(x - conj x) o (rx - a x o (U t))] / b
        double2 vk[4], rk[4];   // the correction's v_k at the lane's subcarriers k = i + 16 m
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const int k = i + 16 * m;
            const int kc = k < NSC ? k : 0;
            double2 x = ld2(a.tx, base + kc);
            const double2 r = ld2(a.rx, base + kc);
            if (!((xm >> kc) & 1ull) || k >= NSC) x = make_double2(0.0, 0.0);
            vk[m] = x;   // (x_k for now; v_k below)
            rk[m] = r;
        }
        double2 uy[4] = {make_double2(0, 0), make_double2(0, 0), make_double2(0, 0), make_double2(0, 0)};
#pragma unroll
        for (int j = 0; j < R; ++j) {   // (U t)_k, t_j broadcast once per j
            const double2 tj = row_bcast_n(t, j);
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const int k = i + 16 * m;
                uy[m] = cadd(uy[m], cmul(UT[j * CLD + (k < NSC ? k : 0)], tj));
            }
        }
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const double2 x = vk[m];
            const double2 rho = csub(rk[m], cscale(cmul(x, uy[m]), ac));
            vk[m] = make_double2(-2.0 * x.y * rho.y, 2.0 * x.y * rho.x);
        }
        const double rb = 1.0 / bc;
#pragma unroll
        for (int j = 0; j < R; ++j) {   // c_j = sum_k conj(U_kj) v_k over the row; lane j keeps t_j + c_j / b
            double2 cp = make_double2(0.0, 0.0);
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const int k = i + 16 * m;
                cp = cadd(cp, cmul(cconj(UT[j * CLD + (k < NSC ? k : 0)]), vk[m]));
            }
            const double2 cj = row16_sum(cp);
            if (i == j) t = cadd(t, cscale(cj, rb));
        }
    }
    double2 y[4];   // H_k = U_k s at k = i + 16 m: t_j broadcast once per j
#pragma unroll
    for (int m = 0; m < 4; ++m) y[m] = make_double2(0.0, 0.0);
    if constexpr (TQ) {   // U[k][j] = s_j E[k j]: the pair-form read-out of mmse_lr_quad2_kernel (round 6)
        const double ts = row ? st->col_s[i] : 0.0;
        double2 c = cscale(t, ts);   // s_i t_i on lane i
        const double2 h0 = row16_sum(c);
        const int k1 = i + 1, k2 = i + 17;
        const bool two = k2 <= NSC / 2;
        const uint32_t s1 = 16u * (uint32_t)k1, w1 = s1 - 16u * NSC;
        const uint32_t s2 = 16u * (uint32_t)(two ? k2 : k1), w2 = s2 - 16u * NSC;
        uint32_t o1 = 0, o2 = 0;
        double2 A1 = make_double2(0.0, 0.0), B1 = A1, A2 = A1, B2 = A1;
        dpp_ready(c);
        lrq2_readout<R, 0>(sE, c, c, o1, o2, s1, w1, s2, w2, A1, B1, A2, B2);
        if (i == 0) st2(W, 0, h0);
        st2(W, k1, make_double2(A1.x - B1.y, A1.y + B1.x));
        st2(W, NSC - k1, make_double2(A1.x + B1.y, A1.y - B1.x));
        if (two) {
            st2(W, k2, make_double2(A2.x - B2.y, A2.y + B2.x));
            st2(W, NSC - k2, make_double2(A2.x + B2.y, A2.y - B2.x));
        }
        return;
    } else {
#pragma unroll
    for (int j = 0; j < R; ++j) {
        const double2 tj = row_bcast_n(t, j);
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const int k = i + 16 * m;
            const double2 u = UT[j * CLD + (k < NSC ? k : 0)];
            y[m].x = fma(u.x, tj.x, fma(-u.y, tj.y, y[m].x));
            y[m].y = fma(u.x, tj.y, fma(u.y, tj.x, y[m].y));
        }
    }
    }
#pragma unroll
    for (int m = 0; m < 4; ++m)   // the row stores 256 B of its frame per m
        if (i + 16 * m < NSC) st2(W, i + 16 * m, y[m]);
}

// H[f] = (((X[4f] + X[4f+1]) + X[4f+2]) + X[4f+3]) / 4  (WiFi_channel_estimation_PS_MMSE.m:35)
__global__ __launch_bounds__(256) void avg_blocks_kernel(const double *__restrict__ X, int64_t xs, double *H, int64_t hs,
                                                         int64_t n)
{
    const int64_t f = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int k = threadIdx.x & 63;
    if (f >= n || k >= NSC) return;
    double2 acc = ld2(X, (4 * f) * xs + k);
#pragma unroll
    for (int b = 1; b < 4; ++b) acc = cadd(acc, ld2(X, (4 * f + b) * xs + k));
    st2(H, f * hs + k, cscale(acc, 0.25));
}

// Config 5 fused: the MMSE solve of one frame, then -- with the wave's
// registers free -- that frame's LS family and equalization from the same
// resident data (pilots from LDS, rx blocks streamed).  The HBM traffic of the
// LS path overlaps the VALU-bound solve instead of running as its own pass.
// C semantics, one block.  FC: per-frame covariance (H written directly).
template <bool R1, bool HOUT, bool EQ>
__global__ __launch_bounds__(64, SOLVE_WAVES_PER_SIMD) void mmse_solve_ls_kernel(const State *__restrict__ st,
                                                                                    SolveArgs a, LsArgs l)
{
    __shared__ SolveLds s;
    const int64_t f = blockIdx.x;
    if (f >= a.n) return;
    const int lane = threadIdx.x;
    const bool act = lane < NSC;
    const int k = act ? lane : 0;
    const double2 wz = solve_block<R1, HOUT>(st, a, s, f * a.fs + (int64_t)a.blk * a.bs, f);
    if constexpr (HOUT) {   // wz = s = w^T X z: H = u s
        if (act) st2(a.w, f * a.ws + lane, cmul(ld2(a.cu, f * a.cs + lane), wz));
    } else {
        if (act) st2(a.w, f * a.ws + lane, wz);
    }
    // ---- LS family + equalization of frame f (main.c:66-146, WiFi_Equalization.m)
    const uint32_t mask = l.mask;
    if (!mask) return;
    const double2 rp = !l.rx_pre ? make_double2(0, 0) : ld2_nt(l.rx_pre, f * l.ps + k);
    const LsLane c = ls_lane(st, l.tx_pre, k);
    // pilot LS from the frame data the solve staged in LDS (pilots are in X in both modes)
    // lane j < 4 divides pilot j once; the four values are broadcast by readlane
    const int pj = lane & 3;
    const int pil = pj == 0 ? WCE_P0 : pj == 1 ? WCE_P1 : pj == 2 ? WCE_P2 : WCE_P3;
    const double2 hp = cdiv(s.rx[pil], s.x[pil]);
    const double2 h0 = readlane_c(hp, 0), h1 = readlane_c(hp, 1), h2 = readlane_c(hp, 2), h3 = readlane_c(hp, 3);
    const double2 hlt = lt_ls_lane<false>(c, l.rx_pre != nullptr, rp, k);
    double2 hlin, hcub, hsnc;
    ps_lane<false>(c, mask, h0, h1, h2, h3, hlin, hcub, hsnc);
    if (act) ls_store<EQ>(l, f, k, mask, hlt, hlin, hcub, hsnc);
}

// Rank-1 covariance (TEXTBOOK / REF shared factors, or WCE_MMSE_FRAME_COV per
// frame): C_f = u_f w_f^T, so H = u_f s with s = w_f^T X z from the second
// bordered row (solve_block<., DOT>) -- no back-substitution, no C W GEMM.
// split (MATLAB): one wave per (frame, block) writes its s_b to dots[g];
// fc_finish averages.
__global__ __launch_bounds__(64, SOLVE_WAVES_PER_SIMD) void mmse_solve_fc_kernel(const State *__restrict__ st,
                                                                                    SolveArgs a)
{
    __shared__ SolveLds s;
    const int64_t g = blockIdx.x;
    const int64_t f = a.split ? g / a.nblk : g;
    const int b = a.split ? (int)(g - f * a.nblk) : 0;
    if (f >= a.n) return;
    const int lane = threadIdx.x;
    const double2 sd = solve_block<true, true>(st, a, s, f * a.fs + (int64_t)(a.blk + b) * a.bs, f);
    if (a.split) {
        if (lane == 0) st2(a.dots, g, sd);
    } else if (lane < NSC) {
        st2(a.w, f * a.ws + lane, cmul(ld2(a.cu, f * a.cs + lane), sd));
    }
}

// H[f] = cu_f * mean_b dots[f*nblk + b]: one wave per frame, lane = subcarrier
__global__ __launch_bounds__(256) void fc_finish_kernel(SolveArgs a, const double *__restrict__ dots, double *H,
                                                        int64_t hs)
{
    const int64_t f = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63;
    if (f >= a.n || lane >= NSC) return;
    double2 acc = make_double2(0.0, 0.0);
    for (int b = 0; b < a.nblk; ++b) acc = cadd(acc, ld2(dots, f * a.nblk + b));
    st2(H, f * hs + lane, cmul(ld2(a.cu, f * a.cs + lane), cscale(acc, 1.0 / a.nblk)));
}

// =====================================================================
// H = C W on f64 MFMA.  v_mfma_f64_16x16x4_f64: lane l supplies
// A[m = l&15][k = l>>4], B[k = l>>4][n = l&15]; D[m = (l>>4) + 4r][n = l&15].
// Here m = frame (16 per tile), k = input subcarrier j, n = output
// subcarrier i; complex = 4 real MFMAs.  W may alias H: every W fragment of a
// tile is loaded before the first store of that tile.
// =====================================================================
constexpr int APPLY_WAVES = 4;

// A 16-frame tile whose every live frame is flagged done (the constant-modulus
// path wrote their H) needs no W loads, MFMAs or stores (wave-uniform).
__device__ __forceinline__ bool tile_done(const uint8_t *__restrict__ skip, int64_t f0, int64_t n, int lane)
{
    if (!skip) return false;
    const int64_t f = f0 + (lane & 15);
    return __ballot(f < n && skip[f] == 0) == 0;
}
// bit m: frame f0 + m of the tile exists and is not flagged done -- one load per
// lane per tile, where a per-store skip[] test waited a round trip per store
__device__ __forceinline__ uint32_t tile_keep(const uint8_t *__restrict__ skip, int64_t f0, int64_t n, int lane)
{
    const int64_t f = f0 + (lane & 15);
    const bool k = f < n && !(skip && skip[f]);
    return (uint32_t)__ballot(k) & 0xffffu;
}

// H = C W (and the per-frame-covariance factors) in the 3M (Gauss) form: three
// real MFMA chains per complex product, P1 = sum Re w Re c, P2 = sum Im w Im c,
// P3 = sum (Re w + Im w)(Re c + Im c); Re = P1 - P2, Im = (P3 - P1) - P2
// (round 3: 473 -> 406 us per 1,048,576 frames, profiles/r03_ab_apply_3m.txt).
// apply_kernel computes output rows 48..52 on v_mfma_f64_4x4x4_4b (the last
// 16-row block holds 5 live rows); matvec_kernel keeps a fourth 16x16x4 block
// (its C comes from L2, and the 4x4 form reads twice as much of it per tile:
// 45.1 vs 41.6 us at 65,536 frames).  (Round 4 retired the 4-product form,
// the per-block C reads, the deferred stores and the 16x16x4 tail of
// apply_kernel: their A/B results are in profiles/r02_ab_apply.txt,
// r03_ab_apply_tail.txt, r03_ab_apply_3m.txt.)
constexpr int APPLY_NT = 3;    // apply_kernel: 16-row output blocks on 16x16x4 (rows 48..52 on 4x4x4)
constexpr int MATVEC_NT = 4;   // matvec_kernel: all 64 rows on 16x16x4

// Y1[f] = M1 X[f] (and Y2[f] = M2 X[f]) for 16-frame tiles; M padded 64 x 64.
// QIN: the input is replaced by (re X - im X, 0) (main.c:188's real "conj").
// NB > 1: the input of frame f is the mean of rows f*NB .. f*NB+NB-1 of X
// (MATLAB's block average, summed in block order like the reference's mean).
template <bool QIN, bool TWO, int NB = 1>
__global__ __launch_bounds__(256) void matvec_kernel(const double *__restrict__ M1, const double *__restrict__ M2,
                                                     const double *X, int64_t xs, double *Y1, double *Y2,
                                                     int64_t ys, int64_t n, const uint8_t *__restrict__ skip)
{
    const int lane = threadIdx.x & 63;
    const int64_t f0 = ((int64_t)blockIdx.x * APPLY_WAVES + (threadIdx.x >> 6)) * 16;
    if (f0 >= n || tile_done(skip, f0, n, lane)) return;
    const int ml = lane & 15, kl = lane >> 4;
    const int64_t fa = f0 + ml;
    double ar[KSTEPS], ai[KSTEPS], nai[KSTEPS];
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s) {
        const int j = 4 * s + kl;
        double2 v = make_double2(0, 0);
        if (fa < n && j < NSC) {
            if constexpr (NB == 1) {
                v = ld2(X, fa * xs + j);
            } else {
#pragma unroll
                for (int b = 0; b < NB; ++b) v = cadd(v, ld2(X, (fa * NB + b) * xs + j));
                v = cscale(v, 1.0 / NB);
            }
        }
        if constexpr (QIN) v = make_double2(v.x - v.y, 0.0);
        ar[s] = v.x; ai[s] = v.y; nai[s] = -v.y;
    }
#pragma unroll
    for (int m = 0; m < (TWO ? 2 : 1); ++m) {
        const double *M = m == 0 ? M1 : M2;
        double *Y = m == 0 ? Y1 : Y2;
#pragma unroll
        for (int nt = 0; nt < MATVEC_NT; ++nt) {
            const int i = 16 * nt + ml;
            v4d accr = {0, 0, 0, 0}, acci = {0, 0, 0, 0};
            if constexpr (!QIN) {   // apply_kernel's chains and order: bit-identical to it
                v4d p1 = {0, 0, 0, 0}, p2 = {0, 0, 0, 0}, p3 = {0, 0, 0, 0};
#pragma unroll
                for (int s = 0; s < KSTEPS; ++s) {
                    const double2 c = ld2(M, i * CLD + 4 * s + kl);   // zero-padded 64 x 64
                    p1 = __builtin_amdgcn_mfma_f64_16x16x4f64(ar[s], c.x, p1, 0, 0, 0);
                    p2 = __builtin_amdgcn_mfma_f64_16x16x4f64(ai[s], c.y, p2, 0, 0, 0);
                    p3 = __builtin_amdgcn_mfma_f64_16x16x4f64(ar[s] + ai[s], c.x + c.y, p3, 0, 0, 0);
                }
                accr = p1 - p2;
                acci = (p3 - p1) - p2;
            } else {
#pragma unroll
                for (int s = 0; s < KSTEPS; ++s) {
                    const int j = 4 * s + kl;
                    const double2 c = ld2(M, i * CLD + j);   // zero-padded 64 x 64
                    accr = __builtin_amdgcn_mfma_f64_16x16x4f64(ar[s], c.x, accr, 0, 0, 0);
                    if constexpr (!QIN) accr = __builtin_amdgcn_mfma_f64_16x16x4f64(nai[s], c.y, accr, 0, 0, 0);
                    acci = __builtin_amdgcn_mfma_f64_16x16x4f64(ar[s], c.y, acci, 0, 0, 0);
                    if constexpr (!QIN) acci = __builtin_amdgcn_mfma_f64_16x16x4f64(ai[s], c.x, acci, 0, 0, 0);
                }
            }
            if (i < NSC) {
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int64_t fr = f0 + kl + 4 * r;
                    if (fr < n && !(skip && skip[fr])) st2(Y, fr * ys + i, make_double2(accr[r], acci[r]));
                }
            }
        }
    }
}

// =====================================================================
// WCE_MMSE_COV, constant-modulus frames (round 4; wce_ctx_set_modulus).
// Ryy = a X C X^H + b I depends on the frame's symbols only through
// P = X^H X = diag |x_k|^2 once the phases are split off, and for PSK frames
// (the reference's BPSK, inputs.h; QPSK) P is the same for every frame.  By
// the push-through identity C X^H (a X C X^H + b I)^-1 = (a C P + b I)^-1 C X^H:
//   H1 = K (conj(x) o rx),   K = (a C P + b I)^-1 C   (State::Kcm, 80-bit host)
// and for non-real x (the .m file applies X, not X^H; b Ryy^-1 rx = rx - a x o H1)
//   H  = H1 + C [(x - conj x) o (rx - a x o H1)] / b,
// the Gram path's correction term (mmse_lr_kernel), formed the same way.
// Per 16-frame tile (one wave), everything in ONE register layout: lane l
// holds frame l & 15 at subcarriers j = 4 s + (l >> 4).  That is the
// v_mfma_f64_16x16x4 B operand (k = j, n = frame) and, with the matrix as the A
// operand (m = output row), also the D layout of the product (row 16 nt + 4 r
// + (l >> 4) = 4 s' + (l >> 4) with s' = 4 nt + r): H1 lands where the
// correction's inputs are, with no transpose.
//  - x, rx loads; the pattern check |x_j|^2 == pcm[j] (the host's fma, bit for
//    bit) on every subcarrier, per frame over its 4 lanes (ballot);
//  - H1 = K (conj x o rx) on MFMA (3M: three real products per complex one);
//  - a non-real frame in the tile (wave-uniform): y2 = (x - conj x) o (rx - a x
//    o H1), H = H1 + (C y2) (1 / b);
//  - H of the matching frames stored; flags[f] = 1 for them, 0 for the others
//    (left to the per-frame kernels, which skip the flagged units).
// =====================================================================
__device__ __forceinline__ void cm_rows3(const double *__restrict__ M, int nt, const double (&yr)[KSTEPS],
                                         const double (&yi)[KSTEPS], int ml, int kl, v4d &hr, v4d &hi)
{
    v4d p1 = {0, 0, 0, 0}, p2 = {0, 0, 0, 0}, p3 = {0, 0, 0, 0};
    const int i = 16 * nt + ml;   // A operand: M[i][4 s + kl]
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s) {
        const double2 c = ld2(M, i * CLD + 4 * s + kl);   // zero-padded 64 x 64
        p1 = __builtin_amdgcn_mfma_f64_16x16x4f64(c.x, yr[s], p1, 0, 0, 0);
        p2 = __builtin_amdgcn_mfma_f64_16x16x4f64(c.y, yi[s], p2, 0, 0, 0);
        p3 = __builtin_amdgcn_mfma_f64_16x16x4f64(c.x + c.y, yr[s] + yi[s], p3, 0, 0, 0);
    }
    hr = p1 - p2;
    hi = (p3 - p1) - p2;
}
// Two launches: cm_real_kernel (below, persistent) checks every frame,
// finishes the tiles whose matching frames are all real (flags 1) and marks
// matching non-real frames 2; cm_cplx_kernel (its own register allocation: the
// correction holds all of H1) finishes the tiles holding a 2, and exits at
// once elsewhere.
__global__ __launch_bounds__(256) void cm_cplx_kernel(const State *__restrict__ st, SolveArgs a,
                                                      uint8_t *__restrict__ flags)
{
    const int lane = threadIdx.x & 63;
    const int64_t f0 = ((int64_t)blockIdx.x * APPLY_WAVES + (threadIdx.x >> 6)) * 16;
    if (f0 >= a.n) return;
    const int ml = lane & 15, kl = lane >> 4;
    const int64_t fa = f0 + ml;
    const bool live = fa < a.n;
    if (__ballot(live && flags[fa] == 2) == 0) return;   // (wave-uniform) nothing left here
    const int64_t base = live ? fa * a.fs + (int64_t)a.blk * a.bs : 0;
    const uint64_t xm = st->xmask;
    const double ac = st->acoef;
    double yr[KSTEPS], yi[KSTEPS];
    bool bad = !live, cplx = false;
    {   // every load of the tile issued before the first use (cm_real_kernel's form;
        // QPSK frames 138 -> 131 us per 65,536, 1.16 -> 1.01 ms per 524,288, profiles/r05_ab_cmq.txt)
        double2 xs[KSTEPS], rs[KSTEPS];
        double pcs[KSTEPS];
#pragma unroll
        for (int s = 0; s < KSTEPS; ++s) {
            const int j = 4 * s + kl, jc = j < NSC ? j : NSC - 1;
            xs[s] = ld2(a.tx, base + jc);
            rs[s] = ld2(a.rx, base + jc);
            pcs[s] = st->pcm[jc];
        }
#pragma unroll
        for (int s = 0; s < KSTEPS; ++s) {
            const int j = 4 * s + kl;
            double2 x = make_double2(0, 0), r = x;
            if (live && j < NSC) {
                x = ((xm >> j) & 1ull) ? xs[s] : make_double2(0, 0);
                r = rs[s];
                bad |= fma(x.x, x.x, x.y * x.y) != pcs[s];
                cplx |= x.y != 0.0;
            }
            yr[s] = fma(x.x, r.x, x.y * r.y);    // conj(x) rx
            yi[s] = fma(x.x, r.y, -x.y * r.x);
        }
    }
    const uint64_t bb = __ballot(bad), cb = __ballot(cplx);
    const uint32_t ok = ~(uint32_t)((bb | (bb >> 16) | (bb >> 32) | (bb >> 48)) & 0xffffu) & 0xffffu;
    const uint32_t cx = (uint32_t)((cb | (cb >> 16) | (cb >> 32) | (cb >> 48)) & 0xffffu) & ok;
    (void)cx;
    if (ok == 0) return;                        // (wave-uniform) no frame of this tile matches
    const bool mine = (ok >> ml) & 1u;
    // non-real symbols in the tile: all of H1 first (it is the correction's input)
    double h1r[16], h1i[16];   // row 4 s + kl at index s (s = 14, 15: padding rows 56..63)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
        v4d hr, hi;
        cm_rows3(st->Kcm, nt, yr, yi, ml, kl, hr, hi);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            h1r[4 * nt + r] = hr[r];
            h1i[4 * nt + r] = hi[r];
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    // y2 = (x - conj x) o (rx - a x o H1): the frame's loads again (L2-resident), all issued first
    {
        double2 xs[KSTEPS], rs[KSTEPS];
#pragma unroll
        for (int s = 0; s < KSTEPS; ++s) {
            const int j = 4 * s + kl, jc = j < NSC ? j : NSC - 1;
            xs[s] = ld2(a.tx, base + jc);
            rs[s] = ld2(a.rx, base + jc);
        }
#pragma unroll
        for (int s = 0; s < KSTEPS; ++s) {
            const int j = 4 * s + kl;
            double2 x = make_double2(0, 0), r = x;
            if (mine && j < NSC) {
                x = ((xm >> j) & 1ull) ? xs[s] : make_double2(0, 0);
                r = rs[s];
            }
            const double2 rho = csub(r, cscale(cmul(x, make_double2(h1r[s], h1i[s])), ac));
            yr[s] = -2.0 * x.y * rho.y;
            yi[s] = 2.0 * x.y * rho.x;
        }
    }
    const double rb = 1.0 / st->bcoef;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
        v4d cr, ci;
        cm_rows3(st->C, nt, yr, yi, ml, kl, cr, ci);
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int s = 4 * nt + r, i = 4 * s + kl;
            if (mine && i < NSC && s < KSTEPS)
                st2(a.w, fa * a.ws + i, make_double2(h1r[s] + cr[r] * rb, h1i[s] + ci[r] * rb));
        }
        __builtin_amdgcn_sched_barrier(0);
    }
    if (kl == 0 && mine) flags[fa] = 1;
}

// =====================================================================
// Synthetic frames: splitmix64 counter RNG keyed by (seed, frame, stream).
// =====================================================================
__device__ __forceinline__ uint64_t mix64(uint64_t x)
{
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
__device__ __forceinline__ double u01(uint64_t h) { return (double)(h >> 11) * (1.0 / 9007199254740992.0); }
// approximately N(0,1): Irwin-Hall of 4 uniforms, unit variance
__device__ __forceinline__ double gauss(uint64_t key)
{
    const double s = u01(mix64(key)) + u01(mix64(key ^ 0x1111)) + u01(mix64(key ^ 0x2222)) + u01(mix64(key ^ 0x3333));
    return (s - 2.0) * 1.7320508075688772;
}

// 802.11 pilot polarity p_0..p_14 (IEEE 802.11-2016 17.3.5.10) and pilot base.
__constant__ double c_polarity[NBLK] = {1, 1, 1, 1, -1, -1, -1, 1, -1, -1, -1, -1, 1, 1, -1};
__constant__ double c_pilot_base[4] = {1, 1, 1, -1};
constexpr int NTAP = 6;

__global__ __launch_bounds__(256) void synth_kernel(SynthArgs a, const double *__restrict__ tx_pre)
{
    const int lane = threadIdx.x & 63;
    const int64_t fl = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    if (fl >= a.n || lane >= NSC) return;
    const int k = lane;
    const uint64_t fg = (uint64_t)(a.first + fl);
    const uint64_t key = mix64(a.seed ^ mix64(fg));
    double2 h;
    if (a.h_shared) {
        h = ld2(a.h_shared, k);
    } else {
        h = make_double2(0, 0);
        double norm = 0;
        for (int t = 0; t < NTAP; t++) norm += exp(-0.5 * t);
        const double g0 = 0.0105 / sqrt(norm);
        for (int t = 0; t < NTAP; t++) {
            const double sc = g0 * exp(-0.25 * t) * 0.7071067811865476;
            const double2 ht = make_double2(sc * gauss(key ^ (0x100 + 2 * t)), sc * gauss(key ^ (0x101 + 2 * t)));
            double sn, cs;
            sincospi(-2.0 * t * (k - 26) / 64.0, &sn, &cs);
            h = cadd(h, cmul(ht, make_double2(cs, sn)));
        }
    }
    const double sig = sqrt(a.ow2 * 0.5);
    int pidx = -1;
#pragma unroll
    for (int pp = 0; pp < 4; pp++) if (k == PILOT[pp]) pidx = pp;
    for (int b = 0; b < NBLK; b++) {
        double tv;
        if (k == 26) tv = 0.0;
        else if (pidx >= 0) tv = a.amp * c_pilot_base[pidx] * c_polarity[b];
        else tv = (mix64(key ^ (0x10000ull + (uint64_t)(b * 64 + k))) & 1) ? a.amp : -a.amp;
        const double2 t = make_double2(tv, 0);
        const uint64_t nk = key ^ (0x40000ull + (uint64_t)(b * 64 + k) * 2);
        const double2 r = cadd(cmul(h, t), make_double2(sig * gauss(nk), sig * gauss(nk ^ 0x5555)));
        const int64_t o = fl * a.fs + (int64_t)b * a.bs + k;
        if (a.tx) st2(a.tx, o, t);
        st2(a.rx, o, r);
    }
    if (a.rx_pre) {
        const double2 tp = ld2(tx_pre, k);
        const uint64_t nk = key ^ 0x80000ull ^ (uint64_t)k;
        const double sp = sig * 0.7071067811865476;
        st2(a.rx_pre, fl * a.ps + k, cadd(cmul(h, tp), make_double2(sp * gauss(nk), sp * gauss(nk ^ 0x5555))));
    }
}


// =====================================================================
// Non-finite guard ("an optional per-frame non-finite bitmap").
// The reference passes NaN through silently -- its literal PS_MMSE returns
// NaN x 53 (main.c:148-212) and its divisions by a zero pilot give
// Inf.  One HBM pass over an output array on the flat element index
// e = 53 f + k (every lane of a load carries one entry);
// only the rare non-finite lanes touch the bitmap, and the lane whose
// atomicOr sets a frame's bit is the one that counts that frame.
// =====================================================================
template <bool F32>
__global__ __launch_bounds__(256) void nonfinite_scan_kernel(const double *__restrict__ H, int64_t stride,
                                                             int64_t f_begin, uint32_t nfr, uint32_t *bits,
                                                             unsigned long long *n_bad)
{
    const uint32_t E = nfr * (uint32_t)NSC;
    for (uint32_t e = blockIdx.x * 256u + threadIdx.x; e < E; e += gridDim.x * 256u) {
        const uint32_t f = e / NSC, k = e - f * NSC;
        const int64_t idx = (f_begin + f) * stride + k;
        double re, im;
        if constexpr (F32) {
            const v2f t = reinterpret_cast<const v2f *>(H)[idx];
            re = t.x;
            im = t.y;
        } else {
            const double2 t = ld2(H, idx);
            re = t.x;
            im = t.y;
        }
        if (!(__builtin_isfinite(re) && __builtin_isfinite(im))) {
            const int64_t fg = f_begin + f;
            const uint32_t bit = 1u << (fg & 31);
            const uint32_t old = atomicOr(&bits[fg >> 5], bit);
            if (!(old & bit) && n_bad) atomicAdd(n_bad, 1ull);
        }
    }
}

// ---------------------------------------------------------------- launchers
static int hip_status(hipError_t e) { return e == hipSuccess ? WCE_OK : WCE_EHIP; }

// A/B kernel variants, process-wide (wce_debug_set_variant): lets one process
// time two kernels on the same buffers, interleaved.  Defaults = the product.
constexpr int LR_FPW = 64;             // mmse_lr_lane_kernel (direct): units per wave at or below LR_FPW_BELOW units
constexpr int64_t LR_FPW_BELOW = 131072;
// mmse_lr_lane_kernel: the LDS-staged form past this many (frame, block) units.  Round 3, with P_k / U shared
// in LDS (LR_STAGED_LDS_P) the staged form wins at every size: 65,536 frames rank 4 52.1 -> 37.2 us,
// 5 63.1 -> 40.8, 6 65.8 -> 46.8, 7 75.4 -> 53.0, 8 68.1 -> 64.4 (before the LDS sharing: rank 4 direct 51.6 vs
// staged ~60 at 65,536, so 98,304 then)
constexpr int64_t LR_STAGE_FROM = 0;
static int g_variant[WCE_VARIANT_COUNT] = {0, 2, 0, 0, 0};
int set_variant(int which, int value)
{
    if (which < 0 || which >= WCE_VARIANT_COUNT || value < 0 || value > 15) return WCE_EINVAL;
    __atomic_store_n(&g_variant[which], value, __ATOMIC_RELAXED);
    return WCE_OK;
}
static inline int variant(int which) { return __atomic_load_n(&g_variant[which], __ATOMIC_RELAXED); }
int variant_value(int which) { return which >= 0 && which < WCE_VARIANT_COUNT ? variant(which) : 0; }

// blocks of 4 waves for a tile kernel: one wave per tile up to the device's
// resident-wave budget (CUs x waves per CU), grid-stride past it
// CU count of the CURRENT device (callers hold a DeviceGuard for the ctx's
// device), cached per device index: one process may drive several GPUs from
// several threads, so the cache is an array of atomics, not one static int.
static int cu_count()
{
    constexpr int kMaxDev = 64;
    static int cache[kMaxDev] = {};
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || dev < 0) dev = 0;
    int *slot = dev < kMaxDev ? &cache[dev] : nullptr;
    int cus = slot ? __atomic_load_n(slot, __ATOMIC_RELAXED) : 0;
    if (cus <= 0) {
        int n = 0;
        cus = hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0 ? n : 256;
        if (slot) __atomic_store_n(slot, cus, __ATOMIC_RELAXED);
    }
    return cus;
}

static int64_t tile_blocks(int64_t tiles, int waves_per_cu)
{
    const int64_t cap = (int64_t)cu_count() * waves_per_cu / LS_WAVES;
    const int64_t need = (tiles + LS_WAVES - 1) / LS_WAVES;
    return need < cap ? need : cap;
}

int launch_ls(const State *st, const LsArgs &a, void *stream)
{
    if (a.n <= 0) return WCE_OK;
    const int64_t groups = (a.n + LS_FRAMES - 1) / LS_FRAMES;     // one wave per LS_FRAMES frames (grid-stride)
    int64_t blocks = (groups + LS_WAVES - 1) / LS_WAVES;
    if (blocks > 256 * 8) blocks = 256 * 8;      // grid-stride the rest
    const bool eq = (a.mask & WCE_EQUALIZE) && a.eq;
    const dim3 g((unsigned)blocks), b(256);
    const bool light = !eq && (a.mask & ~(uint32_t)(WCE_EST_LT_LS | WCE_EST_PS_LINEAR | WCE_EQUALIZE)) == 0;
    // configs[1] (LT_LS / PS_Linear, C semantics): one element per thread;
    // variant 3 routes it through the per-frame LIGHT kernel (the gate's check)
    if (light && !a.matlab && variant(WCE_VARIANT_LS) != 3) {
        for (int64_t f0 = 0, fc = flat_chunk(); f0 < a.n; f0 += fc) {
            const int64_t nf = a.n - f0 < fc ? a.n - f0 : fc;
            const int64_t blocks = (nf * NSC + 255) / 256;
            hipLaunchKernelGGL(ls_elem_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, st, a, f0,
                               (uint32_t)nf);
        }
        return hip_status(hipGetLastError());
    }
    hipStream_t s = (hipStream_t)stream;
    if (a.matlab) {
        if (eq) hipLaunchKernelGGL((ls_kernel<true, true>), g, b, 0, s, st, a);
        else if (light) hipLaunchKernelGGL((ls_kernel<false, true, true>), g, b, 0, s, st, a);
        else hipLaunchKernelGGL((ls_kernel<false, true>), g, b, 0, s, st, a);
    } else {
        if (eq) hipLaunchKernelGGL((ls_kernel<true, false>), g, b, 0, s, st, a);
        else if (light) hipLaunchKernelGGL((ls_kernel<false, false, true>), g, b, 0, s, st, a);
        else hipLaunchKernelGGL((ls_kernel<false, false>), g, b, 0, s, st, a);
    }
    return hip_status(hipGetLastError());
}

int launch_mmse_solve(const State *st, const SolveArgs &a, void *stream)
{
    if (a.mmse_done) return WCE_EINVAL;   // only launch_mmse_solve_ls's REF element path honours it
    if (a.n <= 0) return WCE_OK;
    const int64_t waves = a.split ? a.n * a.nblk : a.n;
    if (waves > 0x7fffffffll) return WCE_EINVAL;
    if (a.hout && !a.cu) return WCE_EINVAL;
    if (a.nblk > 1 && !a.split) return WCE_EINVAL;   // block averaging runs split
    const dim3 g((unsigned)waves), b(64);
    hipStream_t s = (hipStream_t)stream;
    if (a.hout && a.ref_pilots && !a.split) {
        for (int64_t f0 = 0, fc = flat_chunk(); f0 < a.n; f0 += fc) {
            const int64_t nf = a.n - f0 < fc ? a.n - f0 : fc;
            // past the MALL one element per thread (elem), inside it the chunks on a
            // capped grid (flat): 65,536 frames 20.3 / 25.0 us, 131,072 43.1 / 49.2,
            // 262,144 102.7 / 89.3, 1,048,576 380.9 / 338.7 (flat / elem)
            const int v = variant(WCE_VARIANT_REF);
            if (v == 3 || (v == 0 && nf > REF_ELEM_FROM)) {
                hipLaunchKernelGGL(mmse_ref_elem_kernel, dim3((unsigned)((nf * NSC + 255) / 256)), dim3(256), 0, s, st,
                                   a, f0, (uint32_t)nf);
                continue;
            }
            const int64_t chunks = (nf * NSC + FLAT_CHUNK - 1) / FLAT_CHUNK;
            int64_t fb = (chunks + LS_WAVES - 1) / LS_WAVES;
            if (fb > 256 * 8 && v != 2) fb = 256 * 8;
            hipLaunchKernelGGL(mmse_ref_flat_kernel, dim3((unsigned)fb), dim3(256), 0, s, st, a, f0, (uint32_t)nf);
        }
        return hip_status(hipGetLastError());
    }
    if (a.hout) hipLaunchKernelGGL(mmse_solve_fc_kernel, g, b, 0, s, st, a);
    else if (a.cu) hipLaunchKernelGGL(mmse_solve_kernel<true>, g, b, 0, s, st, a);
    else hipLaunchKernelGGL(mmse_solve_kernel<false>, g, b, 0, s, st, a);
    return hip_status(hipGetLastError());
}

// Which low-rank kernel a (rank, units) launch runs: one decision shared by
// launch_mmse_lr and lr_kernel_name (wce_debug_lr_kernel: bench labels, tests)
enum class LrForm { Direct, Staged64, Staged, StagedMW, Quad, Quad2, Wave };
// taps: bit 0 State::cov_taps (a diagonal Rhh: the wave kernel's tap-domain
// Gram), bit 1 State::taps_contig (kept taps 0..r-1: the quad and lane
// kernels' Toeplitz form).  Variant 5 runs the product Gram everywhere (A/B).
static bool lr_taps(int taps) { return (taps & 1) && variant(WCE_VARIANT_LR) != 5; }
static bool lr_contig(int taps) { return (taps & 2) && variant(WCE_VARIANT_LR) != 5; }
static LrForm lr_form(int rank, int64_t units, int taps)
{
    int lv = variant(WCE_VARIANT_LR);
    if (lv >= 5 && lv <= 7) lv = 0;   // 5 changes only the Gram form (lr_taps / lr_contig), 6 / 7 only quad2's build
    if (rank >= 1 && rank <= LRL_RMAX && lv != 1) {
        // the LDS-staged form at every size by default (LR_STAGE_FROM = 0);
        // the direct form runs only as variant 2, the gate's independent check
        // of the staging (tests/test_cov_lowrank_gpu.py)
        const bool staged = lv >= 3 || (lv == 0 && units > LR_STAGE_FROM);
        if (!staged) return LrForm::Direct;
        if (lr_staged_threads(rank) != 256) return LrForm::Staged64;
        // ranks 7, 8: the two-workgroups-per-CU build (MW = LR_STAGED_MINWG)
        // past one 64-unit wave per SIMD; variant 3 forces the MW = 1 build and
        // variant 4 the MW = 2 build at any size, so the gate checks both
        const bool many = lv == 4 || (lv == 0 && units > 64 * 4 * (int64_t)cu_count());
        return rank >= 7 && LR_STAGED_MINWG > 1 && many ? LrForm::StagedMW : LrForm::Staged;
    }
    if (rank > LRL_RMAX && rank <= 16 && lv == 0) return LrForm::Quad;
    // ranks 17..32 with taps 0..r-1: two rows per lane (the Toeplitz Gram only;
    // other covariances keep the wave kernel's product / tap-domain Gram)
    if (rank > 16 && rank <= 32 && lv == 0 && lr_contig(taps)) return LrForm::Quad2;
    return LrForm::Wave;
}


const char *lr_kernel_name(int k0, int rank, int taps, int64_t units)
{
    static const char *lane[2][LRL_RMAX + 1] = {
        {"", "mmse_lr_lane_kernel<1>", "mmse_lr_lane_kernel<2>", "mmse_lr_lane_kernel<3>", "mmse_lr_lane_kernel<4>",
         "mmse_lr_lane_kernel<5>", "mmse_lr_lane_kernel<6>", "mmse_lr_lane_kernel<7>", "mmse_lr_lane_kernel<8>"},
        {"", "mmse_lr_lane_staged_kernel<1>", "mmse_lr_lane_staged_kernel<2>", "mmse_lr_lane_staged_kernel<3>",
         "mmse_lr_lane_staged_kernel<4>", "mmse_lr_lane_staged_kernel<5>", "mmse_lr_lane_staged_kernel<6>",
         "mmse_lr_lane_staged_kernel<7>", "mmse_lr_lane_staged_kernel<8>"}};
    static const char *quad[2][8] = {
        {"mmse_lr_quad_kernel<9>", "mmse_lr_quad_kernel<10>", "mmse_lr_quad_kernel<11>", "mmse_lr_quad_kernel<12>",
         "mmse_lr_quad_kernel<13>", "mmse_lr_quad_kernel<14>", "mmse_lr_quad_kernel<15>", "mmse_lr_quad_kernel<16>"},
        {"mmse_lr_quad_kernel<9, true>", "mmse_lr_quad_kernel<10, true>", "mmse_lr_quad_kernel<11, true>",
         "mmse_lr_quad_kernel<12, true>", "mmse_lr_quad_kernel<13, true>", "mmse_lr_quad_kernel<14, true>",
         "mmse_lr_quad_kernel<15, true>", "mmse_lr_quad_kernel<16, true>"}};
    static const char *quad2[4] = {"mmse_lr_quad2_kernel<20>", "mmse_lr_quad2_kernel<24>", "mmse_lr_quad2_kernel<28>",
                                   "mmse_lr_quad2_kernel<32>"};
    static const char *wave[2][7] = {
        {"mmse_lr_kernel<0>", "mmse_lr_kernel<1>", "mmse_lr_kernel<2>", "mmse_lr_kernel<3>", "mmse_lr_kernel<4>",
         "mmse_lr_kernel<5>", "mmse_lr_kernel<6>"},
        {"mmse_lr_kernel<0, true>", "mmse_lr_kernel<1, true>", "mmse_lr_kernel<2, true>", "mmse_lr_kernel<3, true>",
         "mmse_lr_kernel<4, true>", "mmse_lr_kernel<5, true>", "mmse_lr_kernel<6, true>"}};
    static const char *mw[2][2] = {{"mmse_lr_lane_staged_kernel<7, 2>", "mmse_lr_lane_staged_kernel<8, 2>"},
                                   {"mmse_lr_lane_staged_kernel<7, 2, true>", "mmse_lr_lane_staged_kernel<8, 2, true>"}};
    static const char *lanetq[LRL_RMAX + 1] = {
        "", "mmse_lr_lane_staged_kernel<1, 1, true>", "mmse_lr_lane_staged_kernel<2, 1, true>",
        "mmse_lr_lane_staged_kernel<3, 1, true>", "mmse_lr_lane_staged_kernel<4, 1, true>",
        "mmse_lr_lane_staged_kernel<5, 1, true>", "mmse_lr_lane_staged_kernel<6, 1, true>",
        "mmse_lr_lane_staged_kernel<7, 1, true>", "mmse_lr_lane_staged_kernel<8, 1, true>"};
    static_assert(LR_STAGED_MINWG == 2 || LR_STAGED_MINWG <= 1, "lr_kernel_name spells MW = 2");
    const int r = rank < 1 ? 1 : (rank > LRL_RMAX ? LRL_RMAX : rank);
    switch (lr_form(rank, units, taps)) {
    case LrForm::Direct: return lane[0][r];
    case LrForm::Staged64:
    case LrForm::Staged: return lr_contig(taps) && lr_staged_threads(r) == 256 ? lanetq[r] : lane[1][r];
    case LrForm::StagedMW: return mw[lr_contig(taps) ? 1 : 0][r >= 8 ? 1 : 0];
    case LrForm::Quad: return quad[lr_contig(taps) ? 1 : 0][(rank > 16 ? 16 : rank) - 9];
    case LrForm::Quad2: return quad2[(rank > 32 ? 32 - 17 : rank - 17) / 4];
    default: return k0 >= 0 && k0 <= 6 ? wave[lr_taps(taps) ? 1 : 0][k0] : "";
    }
}

int launch_mmse_lr(const State *st, int k0, int rank, int taps, const SolveArgs &a, void *stream)
{
    if (a.mmse_done) return WCE_EINVAL;
    if (a.n <= 0) return WCE_OK;
    const int64_t waves = a.split ? a.n * a.nblk : a.n;
    if (waves > 0x7fffffffll) return WCE_EINVAL;
    if (a.nblk > 1 && !a.split) return WCE_EINVAL;
    hipStream_t s = (hipStream_t)stream;
    const LrForm form = lr_form(rank, waves, taps);
    if (form == LrForm::Direct || form == LrForm::Staged64 || form == LrForm::Staged || form == LrForm::StagedMW) {
        // direct form: fewer units per wave on a small batch (latency-bound at one wave per SIMD)
        const int fpw = waves <= LR_FPW_BELOW ? LR_FPW : 64;
        const int64_t dw = (waves + fpw - 1) / fpw;
        const dim3 gs((unsigned)((waves + 63) / 64)), bs(64), gd((unsigned)((dw + 3) / 4)), bd(256);
        const dim3 gs4((unsigned)((waves + 255) / 256)), bs4(256);   // staged, 4-wave workgroups (LR_STAGED_LDS_P)
        const bool tq = lr_contig(taps);
#define WCE_LRL(RR)                                                                                         \
    case RR:                                                                                                \
        if constexpr (RR >= 7 && lr_staged_threads(RR) == 256 && LR_STAGED_MINWG > 1) {                \
            if (form == LrForm::StagedMW) {                                                                 \
                if (tq) hipLaunchKernelGGL((mmse_lr_lane_staged_kernel<RR, LR_STAGED_MINWG, true>), gs4, bs4, 0, s, st, a); \
                else hipLaunchKernelGGL((mmse_lr_lane_staged_kernel<RR, LR_STAGED_MINWG>), gs4, bs4, 0, s, st, a); \
                break;                                                                                      \
            }                                                                                               \
        }                                                                                                   \
        if constexpr (lr_staged_threads(RR) == 256) {                                                      \
            if (form == LrForm::Staged && tq) {                                                             \
                hipLaunchKernelGGL((mmse_lr_lane_staged_kernel<RR, 1, true>), gs4, bs4, 0, s, st, a);       \
                break;                                                                                      \
            }                                                                                               \
        }                                                                                                   \
        if (form == LrForm::Staged) hipLaunchKernelGGL(mmse_lr_lane_staged_kernel<RR>, gs4, bs4, 0, s, st, a); \
        else if (form == LrForm::Staged64) hipLaunchKernelGGL(mmse_lr_lane_staged_kernel<RR>, gs, bs, 0, s, st, a); \
        else hipLaunchKernelGGL(mmse_lr_lane_kernel<RR>, gd, bd, 0, s, st, a, fpw);                         \
        break;
        switch (rank) {
            WCE_LRL(1) WCE_LRL(2) WCE_LRL(3) WCE_LRL(4) WCE_LRL(5) WCE_LRL(6) WCE_LRL(7)
            default: WCE_LRL(8)
        }
#undef WCE_LRL
        return hip_status(hipGetLastError());
    }
    if (form == LrForm::Quad) {
        const dim3 gq((unsigned)((waves + 15) / 16)), bq(256);
        const bool tq = lr_contig(taps);
#define WCE_LRQ(RR)                                                                              \
    case RR:                                                                                     \
        if (tq && RR == 16 && variant(WCE_VARIANT_LR) == 6)   /* A/B: separate DPP movs */        \
            hipLaunchKernelGGL((mmse_lr_quad_kernel<16, true, false>), gq, bq, 0, s, st, a);     \
        else if (tq) hipLaunchKernelGGL((mmse_lr_quad_kernel<RR, true>), gq, bq, 0, s, st, a);   \
        else hipLaunchKernelGGL((mmse_lr_quad_kernel<RR, false>), gq, bq, 0, s, st, a);          \
        break;
        switch (rank) {
            WCE_LRQ(9) WCE_LRQ(10) WCE_LRQ(11) WCE_LRQ(12) WCE_LRQ(13) WCE_LRQ(14) WCE_LRQ(15)
            default: WCE_LRQ(16)
        }
#undef WCE_LRQ
        return hip_status(hipGetLastError());
    }
    if (form == LrForm::Quad2) {   // wce_lr_quad2.hip; A/B: variant 6 the Cholesky's broadcasts as separate movs,
        const int lv = variant(WCE_VARIANT_LR);   // 7 every size at 1 wave per SIMD (no spills)
        return launch_lr_quad2(st, rank, a, stream, lv == 6 ? 1 : lv == 7 ? 2 : 0);
    }
    const dim3 g((unsigned)waves), b(64);
    const bool tp = lr_taps(taps);
#define WCE_LRW(K)                                                                               \
    case K:                                                                                      \
        if (tp) hipLaunchKernelGGL((mmse_lr_kernel<K, true>), g, b, 0, s, st, a);                \
        else hipLaunchKernelGGL((mmse_lr_kernel<K, false>), g, b, 0, s, st, a);                  \
        break;
    switch (k0) {
        WCE_LRW(0) WCE_LRW(1) WCE_LRW(2) WCE_LRW(3) WCE_LRW(4) WCE_LRW(5) WCE_LRW(6)
    default: return WCE_EINVAL;
    }
#undef WCE_LRW
    return hip_status(hipGetLastError());
}

int launch_avg_blocks(const double *X, int64_t xs, double *H, int64_t hs, int64_t n, void *stream)
{
    if (n <= 0) return WCE_OK;
    hipLaunchKernelGGL(avg_blocks_kernel, dim3((unsigned)((n + 3) / 4)), dim3(256), 0, (hipStream_t)stream, X, xs, H,
                       hs, n);
    return hip_status(hipGetLastError());
}

int launch_fc_finish(const SolveArgs &a, const double *dots, double *H, int64_t hs, void *stream)
{
    if (a.mmse_done) return WCE_EINVAL;
    if (a.n <= 0) return WCE_OK;
    hipLaunchKernelGGL(fc_finish_kernel, dim3((unsigned)((a.n + 3) / 4)), dim3(256), 0, (hipStream_t)stream, a,
                       dots, H, hs);
    return hip_status(hipGetLastError());
}

int launch_mmse_solve_ls(const State *st, const SolveArgs &a, const LsArgs &l, void *stream)
{
    if (a.n <= 0) return WCE_OK;
    if (a.hout && !a.cu) return WCE_EINVAL;
    if (a.mmse_done && !(a.ref_pilots && a.hout && !a.split && variant(WCE_VARIANT_REF_LS) == 0)) return WCE_EINVAL;
    const dim3 g((unsigned)a.n), b(64);
    hipStream_t s = (hipStream_t)stream;
    const bool eq = (l.mask & WCE_EQUALIZE) && l.eq;
    if (a.ref_pilots && a.hout && !a.split && variant(WCE_VARIANT_REF_LS) == 0) {
        for (int64_t f0 = 0, fc = flat_chunk(); f0 < a.n; f0 += fc) {   // 53 * frames < 2^32 per launch
            const int64_t nf = a.n - f0 < fc ? a.n - f0 : fc;
            const dim3 gb((unsigned)((nf * NSC + 255) / 256));
            if (eq) hipLaunchKernelGGL(ref_ls_elem_kernel<true>, gb, dim3(256), 0, s, st, a, l, f0, (uint32_t)nf);
            else hipLaunchKernelGGL(ref_ls_elem_kernel<false>, gb, dim3(256), 0, s, st, a, l, f0, (uint32_t)nf);
        }
        return hip_status(hipGetLastError());
    }
#define WCE_LAUNCH_SLS(R1, HOUT)                                                                        \
    do {                                                                                                \
        if (eq) hipLaunchKernelGGL((mmse_solve_ls_kernel<R1, HOUT, true>), g, b, 0, s, st, a, l);       \
        else hipLaunchKernelGGL((mmse_solve_ls_kernel<R1, HOUT, false>), g, b, 0, s, st, a, l);         \
    } while (0)
    if (a.hout) WCE_LAUNCH_SLS(true, true);
    else if (a.cu) WCE_LAUNCH_SLS(true, false);
    else WCE_LAUNCH_SLS(false, false);
#undef WCE_LAUNCH_SLS
    return hip_status(hipGetLastError());
}

// H = C W for the dense-C (COV) path, streaming form.  matvec_kernel runs one
// 16-frame tile per wave and one wave round for a whole launch, so every wave
// loads W, multiplies, then stores at the same time: the HBM and MFMA phases
// never overlap.  Here C is staged once per workgroup in LDS (row stride
// ACS = 58 complex, conflict-free: below) and each wave
// walks a strided sequence of 16-frame tiles, loading tile t + 1's W while
// its MFMAs run on tile t.  Same fragment maps and summation order as
// matvec_kernel for rows 0..47; rows 48..52 on v_mfma_f64_4x4x4_4b
// (apply_tile3: 508 -> 465 us per 1,048,576 frames), whose results matched
// the 16x16x4 form bit for bit on every A/B run (tools/ab_libs.py --leg apply).
constexpr int APPLY_WG_PER_CU = 2;
// Row stride (complex) of the staged C.  A read sc[i * ACS + 4 s + kl] (i =
// 16 nt + (lane & 15), kl = lane >> 4) is a ds_read_b128, banked in four
// 16-lane groups {0-3,12-15,20-27}, {4-11,16-19,28-31}, ... on 16-B slots
// (ACS ml + kl) mod 16: ACS = 57 put 3 lanes of a group on one slot (8 LDS
// cycles per read instead of 4: the 3.97 conflict cycles per LDS instruction
// of r02_pmc_legs.json apply1m); 58 maps every group onto 16 distinct slots
// (tools/lds_banks.py enumerates the strides).
constexpr int ACS = 58;
// staged rows of C: 56 (rows 48..55 are the last ones read)
constexpr int APPLY_ROWS = 56;
// A 56 x 56 complex matrix (global rows of stride CLD, zero-padded 64 x 64)
// into LDS rows of stride ACS, and Re + Im beside it when scs: every thread's
// 13 loads issued before its first LDS store.  The plain strided loop waited
// each load before its store, 13 memory round trips at the start of every
// workgroup (profiles/r05_ab_stage.txt).
constexpr int STAGE_N = APPLY_ROWS * 4 * KSTEPS;   // 3,136 elements
constexpr int STAGE_IT = (STAGE_N + 255) / 256;    // 13 per thread of a 256-thread workgroup
__device__ __forceinline__ void stage_load(const double *M, double2 (&v)[STAGE_IT])
{
#pragma unroll
    for (int it = 0; it < STAGE_IT; ++it) {
        const int e = min((int)threadIdx.x + 256 * it, STAGE_N - 1);   // past the end: a valid address, not stored
        const int i = e / (4 * KSTEPS), j = e - i * (4 * KSTEPS);
        v[it] = ld2(M, i * CLD + j);
    }
}
__device__ __forceinline__ void stage_store(const double2 (&v)[STAGE_IT], double2 *sc, double *scs)
{
#pragma unroll
    for (int it = 0; it < STAGE_IT; ++it) {
        const int e = (int)threadIdx.x + 256 * it;
        if (e < STAGE_N) {
            const int i = e / (4 * KSTEPS), j = e - i * (4 * KSTEPS);
            sc[i * ACS + j] = v[it];
            if (scs) scs[i * ACS + j] = v[it].x + v[it].y;
        }
    }
}
__device__ __forceinline__ void apply_load(const double *X, int64_t xs, int64_t n, int64_t g, int ml, int kl,
                                           double2 (&w)[KSTEPS], bool done = false)
{
    const int64_t fa = 16 * g + ml;
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s) {
        const int j = 4 * s + kl;
        w[s] = (!done && fa < n && j < NSC) ? ld2(X, fa * xs + j) : make_double2(0, 0);
    }
}

// One 16-frame tile: rows 0..47 as one flat sequence of 3 x 14 k-steps, C's
// LDS fragments for step t + PF read at step t (PF = 2).  Left to itself the
// compiler issues each k-step's ds_read_b128 right before its MFMAs and waits
// on it (lgkmcnt(0) every few MFMAs), so the MFMA pipe idles for an LDS round
// trip per k-step; a scheduling barrier per step pins every read at its step.
// Each 16-row block's results are stored as soon as they are final.  Rows
// 48..52 on v_mfma_f64_4x4x4_4b: lane l = 16 r + 4 b + c holds A_b[c][r],
// B_b[r][c], D_b[r][c] (profiles/r02_ubench_mfma4.txt); block b = frames
// 4b .. 4b+3, so B_b[k][n] = W_{4b+n}[4s+k] is the W fragment lane l already
// holds for 16x16x4 (frame l&15, subcarrier 4s + (l>>4)); A_b[m][k] =
// C[i0+m][4s+k]; D: lane l gets H_{frame l&15}[i0 + (l>>4)].  Two row groups
// (48..51, 52..55), three independent chains each.  The Gauss form's imaginary
// part carries ~eps (|Re w| + |Im w|)(|Re c| + |Im c|) per term, the same order
// as the 4-product form's ~eps (|Re w Im c| + |Im w Re c|).
// SCS: Re c + Im c staged beside c (apply_kernel); else added per k-step (one
// VALU add, the same bits).  Outputs through the Store: row16(r, i, v) for
// frame kl + 4 r, row4(i, v) for frame ml.
constexpr int APPLY_PF = 2;
template <bool SCS, class Store>
__device__ __forceinline__ void apply_tile3(const double2 *sc, const double *scs, const double (&ar)[KSTEPS],
                                            const double (&ai)[KSTEPS], int ml, int kl, const Store &out)
{
    constexpr int NS = APPLY_NT * KSTEPS;
    constexpr int PF = APPLY_PF;
    double2 cb[PF];
    double cbs[PF];
#pragma unroll
    for (int t = 0; t < PF; ++t) {
        const int e = (16 * (t / KSTEPS) + ml) * ACS + 4 * (t % KSTEPS) + kl;
        cb[t] = sc[e];
        if constexpr (SCS) cbs[t] = scs[e];
    }
    v4d p1 = {0, 0, 0, 0}, p2 = {0, 0, 0, 0}, p3 = {0, 0, 0, 0};
#pragma unroll
    for (int t = 0; t < NS; ++t) {
        const int nt = t / KSTEPS, s = t % KSTEPS;
        const double2 c = cb[t % PF];
        const double cs = SCS ? cbs[t % PF] : c.x + c.y;
        if (t + PF < NS) {
            const int e = (16 * ((t + PF) / KSTEPS) + ml) * ACS + 4 * ((t + PF) % KSTEPS) + kl;
            cb[t % PF] = sc[e];
            if constexpr (SCS) cbs[t % PF] = scs[e];
        }
        const double as = ar[s] + ai[s];
        __builtin_amdgcn_sched_barrier(0);
        p1 = __builtin_amdgcn_mfma_f64_16x16x4f64(ar[s], c.x, p1, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        p2 = __builtin_amdgcn_mfma_f64_16x16x4f64(ai[s], c.y, p2, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        p3 = __builtin_amdgcn_mfma_f64_16x16x4f64(as, cs, p3, 0, 0, 0);
        __builtin_amdgcn_sched_barrier(0);
        if (s == KSTEPS - 1) {
            const v4d hr = p1 - p2, hi = (p3 - p1) - p2;
            const int i = 16 * nt + ml;
            if (i < NSC) {
#pragma unroll
                for (int r = 0; r < 4; ++r) out.row16(r, i, make_double2(hr[r], hi[r]));
            }
            p1 = p2 = p3 = v4d{0, 0, 0, 0};
        }
    }
    const int m4 = ml & 3;
    double a0 = 0.0, b0 = 0.0, g0 = 0.0, a1 = 0.0, b1 = 0.0, g1 = 0.0;
    double2 n0 = sc[(48 + m4) * ACS + kl], n1 = sc[(52 + m4) * ACS + kl];
    double ns0 = 0.0, ns1 = 0.0;
    if constexpr (SCS) {
        ns0 = scs[(48 + m4) * ACS + kl];
        ns1 = scs[(52 + m4) * ACS + kl];
    }
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s) {
        const double2 c0 = n0, c1 = n1;
        const double cs0 = SCS ? ns0 : c0.x + c0.y, cs1 = SCS ? ns1 : c1.x + c1.y;
        asm volatile("" ::: "memory");
        if (s + 1 < KSTEPS) {
            n0 = sc[(48 + m4) * ACS + 4 * (s + 1) + kl];
            n1 = sc[(52 + m4) * ACS + 4 * (s + 1) + kl];
            if constexpr (SCS) {
                ns0 = scs[(48 + m4) * ACS + 4 * (s + 1) + kl];
                ns1 = scs[(52 + m4) * ACS + 4 * (s + 1) + kl];
            }
        }
        const double as = ar[s] + ai[s];
        a0 = __builtin_amdgcn_mfma_f64_4x4x4f64(c0.x, ar[s], a0, 0, 0, 0);
        a1 = __builtin_amdgcn_mfma_f64_4x4x4f64(c1.x, ar[s], a1, 0, 0, 0);
        b0 = __builtin_amdgcn_mfma_f64_4x4x4f64(c0.y, ai[s], b0, 0, 0, 0);
        b1 = __builtin_amdgcn_mfma_f64_4x4x4f64(c1.y, ai[s], b1, 0, 0, 0);
        g0 = __builtin_amdgcn_mfma_f64_4x4x4f64(cs0, as, g0, 0, 0, 0);
        g1 = __builtin_amdgcn_mfma_f64_4x4x4f64(cs1, as, g1, 0, 0, 0);
    }
    out.row4(48 + kl, make_double2(a0 - b0, (g0 - a0) - b0));
    if (kl == 0) out.row4(52, make_double2(a1 - b1, (g1 - a1) - b1));   // rows 53..55: padding, never stored
}

// apply_kernel's stores: H = C W rows of the live, not-skipped frames (tile_keep)
struct ApplyStore {
    double *Y;
    int64_t ys, f0;
    uint32_t keep;   // bit m: frame f0 + m
    __device__ void row16(int r, int i, double2 v) const
    {
        const int m = (threadIdx.x & 63) / 16 + 4 * r;
        if ((keep >> m) & 1u) st2(Y, (f0 + m) * ys + i, v);
    }
    __device__ void row4(int i, double2 v) const
    {
        const int m = threadIdx.x & 15;
        if ((keep >> m) & 1u) st2(Y, (f0 + m) * ys + i, v);
    }
};

__global__ __launch_bounds__(256, APPLY_WG_PER_CU) void apply_kernel(const double *__restrict__ M, const double *X,
                                                                        int64_t xs, double *Y, int64_t ys, int64_t n,
                                                                        const uint8_t *__restrict__ skip)
{
    __shared__ double2 sc[APPLY_ROWS * ACS];
    __shared__ double scs[APPLY_ROWS * ACS];   // Re c + Im c (3M form)
    {
        double2 v[STAGE_IT];
        stage_load(M, v);   // M zero-padded 64 x 64
        stage_store(v, sc, scs);
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int ml = lane & 15, kl = lane >> 4;
    const int64_t ng = (n + 15) / 16;
    const int64_t stride = (int64_t)gridDim.x * APPLY_WAVES;
    int64_t g = (int64_t)blockIdx.x * APPLY_WAVES + (threadIdx.x >> 6);
    if (g >= ng) return;
    double2 wn[KSTEPS];
    uint32_t kn = tile_keep(skip, 16 * g, n, lane);
    apply_load(X, xs, n, g, ml, kl, wn, kn == 0);
    for (; g < ng; g += stride) {
        double ar[KSTEPS], ai[KSTEPS];
#pragma unroll
        for (int s = 0; s < KSTEPS; ++s) {
            ar[s] = wn[s].x;
            ai[s] = wn[s].y;
        }
        const uint32_t keep = kn;
        if (g + stride < ng) {   // next tile, under this one's MFMAs
            kn = tile_keep(skip, 16 * (g + stride), n, lane);
            apply_load(X, xs, n, g + stride, ml, kl, wn, kn == 0);
        }
        if (keep == 0) continue;
        apply_tile3<true>(sc, scs, ar, ai, ml, kl, ApplyStore{Y, ys, 16 * g, keep});
    }
}

// =====================================================================
// REF per-frame covariance (WCE_MMSE_FRAME_COV with WCE_MMSE_REF, C
// semantics).  main.c's PS_MMSE consumes the frame's own H_EST_LT_LS
// (main.c:37-53, 148): g = invF h, Rhh = g q(g)^T, C = F Rhh FH = u w^T with
// u = F invF h = Mu h and w = Mw q(g), and with Ryy = 2 ow2 I and X the 4
// pilots, H = u s, s = sum_p w_p x_p rx_p / b (main.c:186-205).  Only w at
// the pilot rows P = {5, 19, 33, 47} is ever read, and q(g) = re g - im g is
// real-linear in (re h, im h), so w_P = Ar re h + Ai im h with the 4 x 53
// real maps Ar, Ai formed once in 80 bits (State::Wp, round 5): g is never
// formed, and the per-frame MFMA work is the one product u = Mu h.
//
// Lane layout throughout = the MFMA A layout: lane l holds frame l & 15 of
// the 16-frame tile at subcarriers j = 4 s + (l >> 4), s < 14.
//   h    = LT_LS(tx_pre, rx_pre_f)        ls_elem_kernel's formula (main.c:66-75)
//   w_p  = sum over the lane's j, then over the 4 lanes of the frame
//          (ref_w4: 2 x 14 FMA per pilot, permlane16/32 sums)
//   s    = ref_sum4(ref_term(w_p, x_p, rx_p)) / b    the REF kernels' rounding
//   H    = u s, u = Mu h on f64 MFMA           apply_tile3's chains (3M form)
// The variant path (WCE_VARIANT_REF_FC = 1, and MATLAB semantics) forms the
// same values in separate launches (LT_LS pass, matvec of Mu, ref_w_kernel,
// the REF read-out) and is bit-identical to it.
// =====================================================================
__device__ __forceinline__ void ref_w4(const double2 *__restrict__ wp, const double (&ar)[KSTEPS],
                                       const double (&ai)[KSTEPS], int kl, double (&w)[4])
{
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        double acc = 0.0;
#pragma unroll
        for (int s = 0; s < KSTEPS; ++s) {
            const double2 c = wp[p * APPLY_ROWS + 4 * s + kl];   // {Ar, Ai}[p][j], zero past j = 52
            acc = fma(c.x, ar[s], acc);
            acc = fma(c.y, ai[s], acc);
        }
        w[p] = sum_xor32(sum_xor16(acc));   // the frame's 4 lanes, same bits in each
    }
}

// h of frame fa at the lane's subcarriers: LT_LS of its preamble (ls_elem_kernel's
// cdiv, the same bits), zero at DC and past 52
__device__ __forceinline__ void ref_h(const double2 (&rp)[KSTEPS], const double2 *tp, int kl, bool live,
                                      double (&ar)[KSTEPS], double (&ai)[KSTEPS])
{
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s) {   // tp: tx_pre staged in LDS, zero past 52
        const int j = 4 * s + kl;
        const double2 t = tp[j];
        const double cq = t.x - t.y;
        const double2 h = cdiv(make_double2(cq * rp[s].x, cq * rp[s].y), make_double2(cq * t.x, cq * t.y));
        const bool on = live && j < NSC && j != WCE_DC;
        ar[s] = on ? h.x : 0.0;
        ai[s] = on ? h.y : 0.0;
    }
}

// s of frame fa from its 4 pilots (x, rx of block blk), loaded by every lane
// of the frame (the same addresses: one request each), summed in pilot order
// (ref_sum4): the same bits in all four lanes and as the REF read-out kernels.
// (Round 5 A/B, profiles/r05_ab_ref_fc.txt: prefetching the pilots with the
// next tile, or issuing them at the tile's start, was slower every time.  The
// kernel loads and uses them BEFORE it issues the next tile's preamble: after
// those, their wait also covered the next tile's loads (one vmcnt, retired in
// order); with tx_pre staged in LDS instead of 14 branch-guarded global loads
// per tile: 50.6 -> 47.2 us per 65,536 frames, profiles/r05_ab_lat.txt.)
__device__ __forceinline__ double2 ref_s(const double (&w)[4], const SolveArgs &a, int64_t fa, double rb)
{
    if (fa >= a.n) return make_double2(0, 0);
    const int64_t o = fa * a.fs + (int64_t)a.blk * a.bs;
    double2 t[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) t[p] = ref_term(make_double2(w[p], 0.0), ld2(a.tx, o + PILOT[p]), ld2(a.rx, o + PILOT[p]));
    return ref_sum4(t[0], t[1], t[2], t[3], rb);
}

constexpr int FC_WG_PER_CU = 2;
struct RefFcShared {
    double2 sc[APPLY_ROWS * ACS];        // Mu rows 0..55 (apply_kernel's staging, no Re + Im copy)
    double2 wp[4 * APPLY_ROWS];          // {Ar, Ai} at the 4 pilots, j < 56
    double2 s[APPLY_WAVES][16];          // s of each wave's current tile
    double2 tp[APPLY_ROWS];              // tx_pre, zero past 52
};
static_assert(FC_WG_PER_CU * sizeof(RefFcShared) <= 160 * 1024, "two workgroups per CU");

// H = u s of the tile's frames: rows 0..47 frame kl + 4 r, rows 48..52 frame ml
struct RefFcStore {
    double *H;
    int64_t hs, f0, n;
    double2 sv[4], sm;
    __device__ void row16(int r, int i, double2 u) const
    {
        const int64_t fr = f0 + (threadIdx.x & 63) / 16 + 4 * r;
        if (fr < n) st2(H, fr * hs + i, ref_out(u, sv[r]));
    }
    __device__ void row4(int i, double2 u) const
    {
        const int64_t fr = f0 + (threadIdx.x & 15);
        if (fr < n) st2(H, fr * hs + i, ref_out(u, sm));
    }
};

// Persistent: each wave walks 16-frame tiles g, g + stride, ... with the next
// tile's preamble in flight under this tile's work; Mu and Wp staged once per
// workgroup.  UOUT (TEXTBOOK per-frame covariance, C semantics): the same
// LT_LS and u = Mu h (Mu = F conj(F) / 53 there), u stored to a.w (row stride
// a.ws) for the solve, no w / s / read-out -- one launch where the general
// path runs the LT_LS pass and matvec_kernel (bit-identical to them).
template <bool UOUT>
__global__ __launch_bounds__(256, FC_WG_PER_CU) void ref_fc_kernel(const State *__restrict__ st, SolveArgs a,
                                                                   const double *__restrict__ rx_pre, int64_t ps,
                                                                   const double *__restrict__ tx_pre)
{
    __shared__ RefFcShared sh;
    {   // Mu, the pilot-row map and tx_pre in one memory round trip
        const int e = min((int)threadIdx.x, 4 * APPLY_ROWS - 1), p = e / APPLY_ROWS, k = e - p * APPLY_ROWS;
        const double2 wpv = ld2(st->Wp, p * NPAD + k);
        const double2 tpv = ld2(tx_pre ? tx_pre : st->tx_pre, min((int)threadIdx.x, NSC - 1));
        double2 v[STAGE_IT];
        stage_load(st->Mu, v);   // Mu zero-padded 64 x 64
        if (threadIdx.x < 4 * APPLY_ROWS) sh.wp[threadIdx.x] = wpv;
        if (threadIdx.x < APPLY_ROWS) sh.tp[threadIdx.x] = threadIdx.x < NSC ? tpv : make_double2(0, 0);
        stage_store(v, sh.sc, nullptr);
    }
    __syncthreads();
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int ml = lane & 15, kl = lane >> 4;
    const int64_t ng = (a.n + 15) / 16;
    const int64_t stride = (int64_t)gridDim.x * APPLY_WAVES;
    int64_t g = (int64_t)blockIdx.x * APPLY_WAVES + wv;
    if (g >= ng) return;
    const double2 *txp = sh.tp;
    const double rb = 1.0 / st->bcoef;
    // the next tile's preamble at the lane's subcarriers, in flight under this tile's work
    double2 rpn[KSTEPS];
    auto load = [&](int64_t gt) {
        const int64_t fa = 16 * gt + ml;
#pragma unroll
        for (int s = 0; s < KSTEPS; ++s) {
            const int j = 4 * s + kl;
            rpn[s] = (fa < a.n && j < NSC) ? ld2_nt(rx_pre, fa * ps + j) : make_double2(0, 0);
        }
    };
    load(g);
    for (; g < ng; g += stride) {
        const int64_t f0 = 16 * g, fa = f0 + ml;
        const bool live = fa < a.n;
        double ar[KSTEPS], ai[KSTEPS];
        ref_h(rpn, txp, kl, live, ar, ai);
        if constexpr (UOUT) {
            if (g + stride < ng) load(g + stride);   // next tile, under this one's MFMAs
            apply_tile3<false>(sh.sc, nullptr, ar, ai, ml, kl, ApplyStore{a.w, a.ws, f0, tile_keep(nullptr, f0, a.n, lane)});
            continue;
        }
        double w[4];
        ref_w4(sh.wp, ar, ai, kl, w);
        const double2 sfr = ref_s(w, a, fa, rb);
        if (g + stride < ng) load(g + stride);   // next tile, under this one's MFMAs
        RefFcStore out{a.w, a.ws, f0, a.n, {}, sfr};
        if (kl == 0) sh.s[wv][ml] = out.sm;
        wave_lds_sync();
#pragma unroll
        for (int r = 0; r < 4; ++r) out.sv[r] = sh.s[wv][kl + 4 * r];
        wave_lds_sync();   // the next tile rewrites sh.s[wv]
        apply_tile3<false>(sh.sc, nullptr, ar, ai, ml, kl, out);
    }
}

// The variant path's w: full rows of w (zero off the pilots) from the frames'
// h rows, ref_w4's arithmetic and lanes (one 16-frame tile per wave)
__global__ __launch_bounds__(256) void ref_w_kernel(const State *__restrict__ st, const double *__restrict__ X,
                                                    int64_t xs, double *W, int64_t ws, int64_t n)
{
    __shared__ double2 wp[4 * APPLY_ROWS];
    for (int e = threadIdx.x; e < 4 * APPLY_ROWS; e += 256) {
        const int p = e / APPLY_ROWS, k = e - p * APPLY_ROWS;
        wp[e] = ld2(st->Wp, p * NPAD + k);
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int64_t f0 = ((int64_t)blockIdx.x * APPLY_WAVES + (threadIdx.x >> 6)) * 16;
    if (f0 >= n) return;
    const int ml = lane & 15, kl = lane >> 4;
    const int64_t fa = f0 + ml;
    double ar[KSTEPS], ai[KSTEPS];
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s) {
        const int j = 4 * s + kl;
        const double2 v = (fa < n && j < NSC) ? ld2(X, fa * xs + j) : make_double2(0, 0);
        ar[s] = v.x;
        ai[s] = v.y;
    }
    double w[4];
    ref_w4(wp, ar, ai, kl, w);
    if (fa >= n) return;
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s) {
        const int j = 4 * s + kl;
        if (j >= NSC) continue;
        const int p = j == WCE_P0 ? 0 : j == WCE_P1 ? 1 : j == WCE_P2 ? 2 : j == WCE_P3 ? 3 : -1;
        st2(W, fa * ws + j, make_double2(p >= 0 ? w[p < 0 ? 0 : p] : 0.0, 0.0));
    }
}

// The constant-modulus operator's real-symbol pass (round 4's cm_kernel<false>),
// persistent: K staged once per workgroup in LDS as apply_kernel stages C
// (plus Re + Im, 3M form), each wave walking 16-frame tiles.  Per tile: x, rx
// loads, the |x|^2 pattern check and flags, y = conj(x)
// o rx in the MFMA A layout, H = K y for the matching frames of tiles whose
// matching frames are all real (apply_tile3: rows 48..52 on 4x4x4); tiles with
// a matching non-real frame are left to cm_cplx_kernel.
struct CmStore {
    double *H;
    int64_t hs, f0;
    uint32_t ok;   // bit m: frame f0 + m matches the pattern
    __device__ void row16(int r, int i, double2 v) const
    {
        const int m = (threadIdx.x & 63) / 16 + 4 * r;
        if ((ok >> m) & 1u) st2(H, (f0 + m) * hs + i, v);
    }
    __device__ void row4(int i, double2 v) const
    {
        const int m = threadIdx.x & 15;
        if ((ok >> m) & 1u) st2(H, (f0 + m) * hs + i, v);
    }
};
// (Round 5 A/B, profiles/r05_ab_cm.txt: the next tile's loads prefetched spill
// at 2 workgroups per CU and lose at 1.)
__global__ __launch_bounds__(256, APPLY_WG_PER_CU) void cm_real_kernel(const State *__restrict__ st, SolveArgs a,
                                                                      uint8_t *__restrict__ flags)
{
    __shared__ double2 sc[APPLY_ROWS * ACS];
    __shared__ double scs[APPLY_ROWS * ACS];   // Re k + Im k (3M form)
    __shared__ double spcm[APPLY_ROWS];        // the |x|^2 pattern, j < 56
    {
        const double pc = st->pcm[threadIdx.x & (NPAD - 1)];
        double2 v[STAGE_IT];
        stage_load(st->Kcm, v);   // Kcm zero-padded 64 x 64
        if (threadIdx.x < APPLY_ROWS) spcm[threadIdx.x] = pc;
        stage_store(v, sc, scs);
    }
    __syncthreads();
    const int lane = threadIdx.x & 63;
    const int ml = lane & 15, kl = lane >> 4;
    const int64_t ng = (a.n + 15) / 16;
    const int64_t stride = (int64_t)gridDim.x * APPLY_WAVES;
    const uint64_t xm = st->xmask;
    for (int64_t g = (int64_t)blockIdx.x * APPLY_WAVES + (threadIdx.x >> 6); g < ng; g += stride) {
        const int64_t f0 = 16 * g, fa = f0 + ml;
        const bool live = fa < a.n;
        const int64_t base = live ? fa * a.fs + (int64_t)a.blk * a.bs : 0;
        double yr[KSTEPS], yi[KSTEPS];
        bool bad = !live, cplx = false;
        {   // every load of the tile issued before the first use: one memory round trip
            // (loads under a per-step branch waited one by one: 14 round trips per tile;
            // 67 -> 63 us per 65,536 frames, 990 -> 863 us per 1,048,576, profiles/r05_ab_lat.txt)
            double2 xs[KSTEPS], rs[KSTEPS];
#pragma unroll
            for (int s = 0; s < KSTEPS; ++s) {
                const int j = 4 * s + kl, jc = j < NSC ? j : NSC - 1;   // clamped: a valid address, never used
                xs[s] = ld2(a.tx, base + jc);
                rs[s] = ld2(a.rx, base + jc);
            }
#pragma unroll
            for (int s = 0; s < KSTEPS; ++s) {
                const int j = 4 * s + kl;
                const bool on = live && j < NSC;
                double2 x = make_double2(0, 0), r = x;
                if (on) {
                    x = ((xm >> j) & 1ull) ? xs[s] : make_double2(0, 0);
                    r = rs[s];
                    bad |= fma(x.x, x.x, x.y * x.y) != spcm[j];
                    cplx |= x.y != 0.0;
                }
                yr[s] = fma(x.x, r.x, x.y * r.y);    // conj(x) rx
                yi[s] = fma(x.x, r.y, -x.y * r.x);
            }
        }
        const uint64_t bb = __ballot(bad), cb = __ballot(cplx);
        const uint32_t ok = ~(uint32_t)((bb | (bb >> 16) | (bb >> 32) | (bb >> 48)) & 0xffffu) & 0xffffu;
        const uint32_t cx = (uint32_t)((cb | (cb >> 16) | (cb >> 32) | (cb >> 48)) & 0xffffu) & ok;
        if (kl == 0 && live) flags[fa] = !((ok >> ml) & 1u) ? 0 : (cx != 0 ? 2 : 1);
        if (ok == 0 || cx != 0) continue;        // (wave-uniform) nothing to do / cm_cplx_kernel's tile
        apply_tile3<true>(sc, scs, yr, yi, ml, kl, CmStore{a.w, a.ws, f0, ok});
    }
}

int launch_mmse_apply(const State *st, const double *W, double *H, int64_t stride, int64_t n, void *stream,
                      const uint8_t *skip)
{
    if (n <= 0) return WCE_OK;
    // the streaming kernel at every size (round 5, profiles/r05_ab_apply.txt:
    // 65,536 frames 39.0 -> 34.5 us against one tile per wave of matvec_kernel,
    // bit-identical; round 2's opposite finding predates the 4x4x4 tail rows)
    const int64_t tiles = (n + 15) / 16;
    static_assert(APPLY_WAVES == LS_WAVES, "tile_blocks counts LS_WAVES waves per workgroup");
    const int64_t blocks = tile_blocks(tiles, APPLY_WAVES * APPLY_WG_PER_CU);
    hipLaunchKernelGGL(apply_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, st->C, W, stride, H,
                       stride, n, skip);
    return hip_status(hipGetLastError());
}

int launch_matvec_avg(const double *M, const double *X, int64_t xs, int nb, double *Y, int64_t ys, int64_t n,
                      void *stream)
{
    if (n <= 0) return WCE_OK;
    if (nb != 4) return WCE_EINVAL;   // MATLAB semantics averages blocks 1..4
    const int64_t blocks = (n + 16 * APPLY_WAVES - 1) / (16 * APPLY_WAVES);
    hipLaunchKernelGGL((matvec_kernel<false, false, 4>), dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream,
                       M, nullptr, X, xs, Y, nullptr, ys, n, (const uint8_t *)nullptr);
    return hip_status(hipGetLastError());
}

int launch_matvec(const double *M1, const double *M2, const double *X, int64_t xs, double *Y1, double *Y2,
                  int64_t ys, int64_t n, bool qin, void *stream)
{
    if (n <= 0) return WCE_OK;
    const int64_t blocks = (n + 16 * APPLY_WAVES - 1) / (16 * APPLY_WAVES);
    const dim3 g((unsigned)blocks), b(256);
    hipStream_t s = (hipStream_t)stream;
    if (qin && M2) return WCE_EINVAL;
    const uint8_t *none = nullptr;
    if (qin) hipLaunchKernelGGL((matvec_kernel<true, false>), g, b, 0, s, M1, M2, X, xs, Y1, Y2, ys, n, none);
    else if (M2) hipLaunchKernelGGL((matvec_kernel<false, true>), g, b, 0, s, M1, M2, X, xs, Y1, Y2, ys, n, none);
    else hipLaunchKernelGGL((matvec_kernel<false, false>), g, b, 0, s, M1, M2, X, xs, Y1, Y2, ys, n, none);
    return hip_status(hipGetLastError());
}

int launch_ref_fc(const State *st, const SolveArgs &a, const double *rx_pre, int64_t ps, const double *tx_pre,
                  void *stream)
{
    if (a.mmse_done) return WCE_EINVAL;
    if (a.n <= 0) return WCE_OK;
    if (a.split || !rx_pre || !a.w) return WCE_EINVAL;
    const int64_t blocks = tile_blocks((a.n + 15) / 16, APPLY_WAVES * FC_WG_PER_CU);
    hipLaunchKernelGGL(ref_fc_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, st, a, rx_pre,
                       ps, tx_pre);
    return hip_status(hipGetLastError());
}

int launch_fc_u(const State *st, const double *rx_pre, int64_t ps, const double *tx_pre, double *U, int64_t us,
                int64_t n, void *stream)
{
    if (n <= 0) return WCE_OK;
    if (!rx_pre || !U) return WCE_EINVAL;
    SolveArgs a{};
    a.n = n;
    a.w = U;
    a.ws = us;
    const int64_t blocks = tile_blocks((n + 15) / 16, APPLY_WAVES * FC_WG_PER_CU);
    hipLaunchKernelGGL(ref_fc_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, st, a, rx_pre,
                       ps, tx_pre);
    return hip_status(hipGetLastError());
}

int launch_ref_w(const State *st, const double *X, int64_t xs, double *W, int64_t ws, int64_t n, void *stream)
{
    if (n <= 0) return WCE_OK;
    const int64_t blocks = (n + 16 * APPLY_WAVES - 1) / (16 * APPLY_WAVES);
    hipLaunchKernelGGL(ref_w_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, st, X, xs, W, ws, n);
    return hip_status(hipGetLastError());
}

int launch_cm(const State *st, const SolveArgs &a, uint8_t *flags, void *stream)
{
    if (a.mmse_done) return WCE_EINVAL;
    if (a.n <= 0) return WCE_OK;
    if (a.split || !flags) return WCE_EINVAL;
    const int64_t blocks = (a.n + 16 * APPLY_WAVES - 1) / (16 * APPLY_WAVES);
    const int64_t pb = tile_blocks((a.n + 15) / 16, APPLY_WAVES * APPLY_WG_PER_CU);
    hipLaunchKernelGGL(cm_real_kernel, dim3((unsigned)pb), dim3(256), 0, (hipStream_t)stream, st, a, flags);
    hipLaunchKernelGGL(cm_cplx_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, st, a, flags);
    return hip_status(hipGetLastError());
}

int launch_synth(const State *st, const SynthArgs &a, void *stream)
{
    if (a.n <= 0) return WCE_OK;
    const int64_t blocks = (a.n + 3) / 4;
    hipLaunchKernelGGL(synth_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, a, st->tx_pre);
    return hip_status(hipGetLastError());
}

int launch_nonfinite_scan(const double *H, int64_t stride, int64_t n, bool f32, uint32_t *bits,
                          unsigned long long *n_bad, void *stream)
{
    hipStream_t s = (hipStream_t)stream;
    if (hipMemsetAsync(bits, 0, (size_t)((n + 31) / 32) * sizeof(uint32_t), s) != hipSuccess) return WCE_EHIP;
    if (n_bad && hipMemsetAsync(n_bad, 0, sizeof(*n_bad), s) != hipSuccess) return WCE_EHIP;
    for (int64_t f0 = 0, fc = flat_chunk(); f0 < n; f0 += fc) {   // fc % 32 == 0: words never straddle launches
        const int64_t nf = n - f0 < fc ? n - f0 : fc;
        int64_t blocks = (nf * NSC + 255) / 256;
        if (blocks > 256 * 8) blocks = 256 * 8;
        if (f32)
            hipLaunchKernelGGL(nonfinite_scan_kernel<true>, dim3((unsigned)blocks), dim3(256), 0, s, H, stride, f0,
                               (uint32_t)nf, bits, n_bad);
        else
            hipLaunchKernelGGL(nonfinite_scan_kernel<false>, dim3((unsigned)blocks), dim3(256), 0, s, H, stride, f0,
                               (uint32_t)nf, bits, n_bad);
    }
    return hip_status(hipGetLastError());
}

}  // namespace wce
