// wce_internal.h -- layout shared by the host code (g++ / hipcc) and the
// gfx950 kernels.  Not part of the public ABI (include/wce.h is).
#pragma once
#include <mutex>
#include <stdint.h>
#include <stddef.h>
#include "../../include/wce.h"

namespace wce {

constexpr int NSC = WCE_NSC;      // 53 useful subcarriers (utils.h:13)
constexpr int NBLK = WCE_NBLK;    // 15 OFDM blocks (utils.h:15)
constexpr int NPAD = 64;          // one wave64 lane per subcarrier
constexpr int CLD = 64;           // leading dimension of the zero-padded C (64 x 64)
constexpr int PILOT[4] = {WCE_P0, WCE_P1, WCE_P2, WCE_P3};
constexpr int32_t STATE_MAGIC = 0x80211;
constexpr int32_t STATE_LAYOUT = 9;   // State layout version: bump with every change to struct State
constexpr int COV_K0_MAX = 6;    // WCE_MMSE_COV low-rank path: last block row a Gram system can start at

// The frame-independent shared state: everything one rank broadcasts to the
// others (one RCCL broadcast of sizeof(State) = wce_state_size() bytes, 371,632 B).
// Complex values are {re, im} fp64.
constexpr int LRL_RMAX = 8;                          // ranks on the lane-per-frame low-rank kernel
constexpr int LRL_NP = LRL_RMAX * (LRL_RMAX + 1) / 2;  // packed lower-triangle entries of its Gram matrix
struct State {
    double C[CLD * CLD * 2];   // MMSE covariance operator, row-major, zero-padded to 64 x 64
                               // (65,536 B): kernels index it without bounds checks
    // Per-frame covariance (WCE_MMSE_FRAME_COV): C_f = u_f w_f^T is rank 1 in
    // both modes, with u_f = Mu h the batched matrix-vector product of the
    // frame's own H_LT (padded 64 x 64, row-major, applied on MFMA):
    //   REF      Mu = F invF_ref (main.c:186-203); w_f is needed at the 4
    //            pilots only and comes from the folded real map Wp below
    //   TEXTBOOK Mu = F conj(F) / 53 (ifft then F), w = conj(u)
    double Mu[CLD * CLD * 2];
    // REF: w at the 4 pilot rows folded into one real map of h (round 5):
    // main.c forms g = invF_ref h, q = re g - im g and w = Mw q with
    // Mw[j][c] = re F[j][c] - im F[j][c]; here
    // w_p = sum_k Ar[p][k] re h_k + Ai[p][k] im h_k with Ar = Mw_P (re invF - im invF),
    // Ai = -Mw_P (re invF + im invF), products in 80 bits (Mw_P = rows P of Mw),
    // so the fold rounds once where main.c rounds per step: parity with main.c
    // is held by tolerance (1e-15 of scale on w, 1e-10 on H), not bitwise.
    // Stored {Ar, Ai} pairs, Wp[2 (p NPAD + k)], zero past k = 52.
    double Wp[4 * NPAD * 2];
    double cvec[NPAD * 2];     // rank-1 factors of the shared C = u w^T: u = cvec and
    double cwvec[NPAD * 2];    // w = conj(cvec) (TEXTBOOK: c = F ifft(H_LT)) or w = cwvec
                               // (REF: u = F g, w = FH^T q, main.c:186-203)
    double h_lt[NPAD * 2];     // LT_LS of the shared preamble (main.c:66-75)
    double tx_pre[NPAD * 2];   // shared tx preamble FFT
    double sinc[4][NPAD];      // sinc((k - P_p)/14) in double (utils.c:727-733)
    double acoef, bcoef;       // Ryy = a X C X' + b I
    double ow2;                // noise variance (inputs.h:18)
    uint64_t xmask;            // bit k set: subcarrier k enters X
    int32_t mode;              // WCE_MMSE_REF / WCE_MMSE_TEXTBOOK / WCE_MMSE_COV
    int32_t magic;             // STATE_MAGIC once valid
    // WCE_MMSE_COV low-rank factor (wce_state_build_cov): C = U U^H with
    // U = F V_r sqrt(Lambda_r) from the 80-bit eigendecomposition of Rhh,
    // zero-padded to 64 x 64 (U[k][j], k = subcarrier, j = eigen-direction),
    // and its transpose UT[j][k].  cov_k0 >= 0: the per-frame solve runs the
    // Gram system (a G^H G + b I) t = G^H rx, G = X U, embedded at block row
    // cov_k0 of the register layout (mmse_lr_kernel); -1: the dense Ryy solve.
    double U[CLD * CLD * 2];
    double UT[CLD * CLD * 2];
    double cov_lmax, cov_lmin; // largest / smallest kept eigenvalue of C
    int32_t cov_rank;          // r = number of kept eigen-directions (0..53)
    int32_t cov_k0;            // -1 dense; else first block row of the embedded Gram system
    int32_t layout;            // STATE_LAYOUT of the build that wrote it
    int32_t bytes;             // sizeof(State) of the build that wrote it
    int32_t reserved[2];       // zero (keeps Pk 16-B aligned)
    // Ranks 1..LRL_RMAX (mmse_lr_lane_kernel): the Gram matrix is sum_k |x_k|^2 P_k
    // with P_k[i][j] = conj(U[k][i]) U[k][j], i >= j, packed at i (i + 1) / 2 + j
    // (80-bit products rounded once; zero for other ranks)
    double Pk[NSC * LRL_NP * 2];
    // WCE_MMSE_COV, constant-modulus frames (wce_ctx_set_modulus, round 4): for
    // frames whose |x_k|^2 equals pcm[k] on every subcarrier, P = diag(pcm) is
    // frame-independent and so is K = (a C P + b I)^-1 C (80-bit, host), and
    // H = K (conj(x) o rx) [+ C ((x - conj x) o (rx - a x o H1)) / b].
    double Kcm[CLD * CLD * 2];
    double pcm[NPAD];
    int32_t cm_on;
    int32_t cm_reserved[3];
    // WCE_MMSE_COV with a diagonal Rhh -- a power-delay profile (round 4): C
    // itself is then the exact-DFT circulant C_ij = sum_t p_t E[(i - j) t] (the
    // model every COV path of such a state evaluates: State::C, U, K).  C's
    // eigen-directions are DFT columns, U[:, j] = s_j F[:, t_j], and the Gram
    // matrix U^H P U (P = diag |x|^2) is s_i s_j Q(t_i - t_j) with Q the DFT of
    // |x|^2: the tap-domain form of the Gram path (mmse_lr_kernel<K0, true>)
    // builds it from 53 per-lane sums instead of the 53 x 53 x 53 product.
    // It runs the exact DFT (dft[], from an 80-bit angle), not main.c's cexp of
    // a double angle (phase error <= 6e-14): the two models' answers differ by
    // <= 1.3e-13 norm-relative on the widest PDP (profiles/r04_accuracy_probe.txt).
    int32_t cov_taps;          // 1: Rhh is diagonal and the tables below are set
    int32_t taps_contig;       // 1: ... and its kept taps are 0..r-1, column j = tap j
    int32_t taps_reserved[2];
    int32_t tap_of[NPAD];      // Gram column j -> delay tap t_j (j < cov_rank; 0 past it)
    int32_t col_of[NPAD];      // delay tap t -> Gram column (-1: dropped, or t >= 53)
    double col_s[NPAD];        // sqrt(lambda_j) by Gram column (0 past cov_rank)
    double tap_s[NPAD];        // sqrt(lambda_t) by tap (0 where col_of is -1)
    double dft[NPAD * 2];      // E[m] = exp(-2 pi i m / 53), m < 53 (0 past it)
};
static_assert(sizeof(State) % 16 == 0, "State must keep 16-B alignment");

// A state blob this build can use: magic, layout version and size of this
// build, a known mode, and (WCE_MMSE_COV) a rank and solve form in range.
// Blobs arrive from other ranks or callers (wce_ctx_load_state,
// wce_state_validate, wce_ctx_mark_ready after a broadcast).
inline bool taps_ok(const State *st)
{
    if (st->cov_taps == 0) return st->taps_contig == 0;
    if (st->cov_taps != 1 || (st->taps_contig != 0 && st->taps_contig != 1)) return false;
    for (int j = 0; j < NPAD; j++) {   // the kernels index LDS tables with these
        if (st->tap_of[j] < 0 || st->tap_of[j] >= NSC) return false;
        if (st->col_of[j] < -1 || st->col_of[j] >= st->cov_rank || (j >= NSC && st->col_of[j] != -1)) return false;
        if (st->taps_contig && j < st->cov_rank && st->tap_of[j] != j) return false;
    }
    return true;
}
inline bool state_ok(const State *st)
{
    if (st->magic != STATE_MAGIC || st->layout != STATE_LAYOUT || st->bytes != (int32_t)sizeof(State)) return false;
    if (st->mode != WCE_MMSE_REF && st->mode != WCE_MMSE_TEXTBOOK && st->mode != WCE_MMSE_COV) return false;
    if (st->mode == WCE_MMSE_COV)
        return st->cov_rank >= 0 && st->cov_rank <= NSC && st->cov_k0 >= -1 && st->cov_k0 <= COV_K0_MAX &&
               (st->cov_k0 >= 0 || st->cov_rank == NSC) &&
               // the Gram kernels' row bound: RMAX = 53 - 8 K0 (lr_solve_taps reads z[8 K0 + col], col < rank)
               (st->cov_k0 < 0 || st->cov_rank <= NSC - 8 * st->cov_k0) && taps_ok(st);
    return st->cov_k0 == -1;
}

// Host-side builders (wce_state.cpp, compiled by g++ for x87 long double).
// `ldc` = long double _Complex as {re, im} pairs of long double.
struct ldc { long double re, im; };

// F[t][f] = cexp(-2*I*PI*t*f/53) exactly as main.c:18-26 evaluates it.
void host_fmatrix(ldc *F);
// The reference's adjugate inverse (utils.c:141-170 / 440-459 / 543-569) in
// 80-bit arithmetic, cofactors spread over threads.
void host_inverse_cofactor(const ldc *A, int n, ldc *Y, int nthreads);
// Cached inverse of the standard F (computed once per process).
const ldc *host_reference_invF();
const ldc *host_reference_F();
// main.c:66-75 in long double.
void host_lt_ls(const ldc *tx_pre, const ldc *rx_pre, ldc *H);
// Fill a host State from F / invF / H_LS (long double) for `mode`.
int host_apply_cov(State *st, const ldc *F, const wce_complex *Rhh);
// WCE_MMSE_COV constant-modulus operator K = (a C P + b I)^-1 C, P = diag(|x_ref|^2)
// (x_ref null: off), from the same Rhh the state was built with
int host_build_cm(State *st, const ldc *F, const wce_complex *Rhh, const wce_complex *x_ref);
int host_build_state(State *st, const ldc *F, const ldc *invF, const ldc *H_LS,
                     const ldc *tx_pre, double ow2, int mode);

// Kernel launchers (wce_kernels.hip).
struct LsArgs {
    const double *tx, *rx, *rx_pre, *tx_pre;
    int64_t fs, bs, ps, n;
    int32_t blk;
    uint32_t mask;
    int32_t matlab;
    int32_t f32;              // WCE_OUT_LS_F32: outputs are complex float
    double *lt, *lin, *cub, *snc, *eq;
    int64_t os, eqfs, eqbs;
    uint32_t eq_src;
    uint32_t pad;
};
struct SolveArgs {
    const double *tx, *rx;
    int64_t fs, bs, n;
    int32_t blk;
    int32_t nblk;             // blocks averaged per frame (1; 4 in MATLAB semantics)
    double *w;
    int64_t ws;
    // rank-1 covariance (null = dense State::C): C_f = cu_f cw_f^T, rows of
    // stride cs (0: one shared pair); cw == null: cw_f = conj(cu_f).
    const double *cu, *cw;
    int64_t cs;
    int32_t hout;             // 1: write H = cu (cw . W) directly (no apply step)
    int32_t split;            // MATLAB averaging: nblk waves per frame, wave g = f*nblk + b
                              // writes W_b to w[g*ws] (or, with hout, cw . W_b to dots[g])
    double *dots;
    int32_t ref_pilots;       // REF (main.c): a = 0 and X = the 4 pilots -> mmse_ref_flat_kernel
    int32_t mmse_done;        // H already written (REF frame covariance): the fused launch runs the LS family only.
                              // Honoured ONLY by launch_mmse_solve_ls's REF element path (ref_ls_elem_kernel);
                              // every other SolveArgs launcher returns WCE_EINVAL when it is set
    const uint8_t *skip;      // per unit: nonzero = H already written (constant-modulus path); null = none
};
struct SynthArgs {
    double *tx, *rx, *rx_pre;
    int64_t fs, bs, ps, first, n;
    uint64_t seed;
    const double *h_shared;
    double amp, ow2;
};

// time-domain front end: unit u = (frame u / nb, unit u % nb); unit samples
// start at src[f*ps + off + 80*b] (complex); bins at dst[f*fs + b*bs + i]
struct FrontArgs {
    const double *src;
    double *dst;
    double *ow2;          // preamble only, may be null
    int64_t ps, off, fs, bs;
    uint32_t n_units, nb;
};

int launch_ls(const State *st, const LsArgs &a, void *stream);
int launch_front(const FrontArgs &a, bool preamble, void *stream);
int launch_mmse_solve(const State *st, const SolveArgs &a, void *stream);
// solve + LS family + equalization of each frame in one launch (C semantics, one block)
int launch_mmse_solve_ls(const State *st, const SolveArgs &a, const LsArgs &l, void *stream);
int launch_mmse_apply(const State *st, const double *W, double *H, int64_t stride, int64_t n, void *stream,
                      const uint8_t *skip = nullptr);
// constant-modulus frames of a WCE_MMSE_COV batch (C semantics): H = K (conj x o rx)
// (+ the correction for non-real x) for every frame whose |x|^2 matches State::pcm;
// flags[f] = 1 for those frames, 0 for the others (left to the per-frame path)
int launch_cm(const State *st, const SolveArgs &a, uint8_t *flags, void *stream);
// Y1[f] = M1 X[f] (and Y2[f] = M2 X[f] if M2), M = padded 64 x 64 complex;
// qin: X replaced by (re X - im X, 0) first.
int launch_matvec(const double *M1, const double *M2, const double *X, int64_t xs, double *Y1, double *Y2,
                  int64_t ys, int64_t n, bool qin, void *stream);
// Y[f] = M mean_b X[f*nb + b]  (MATLAB block average folded into the apply)
int launch_matvec_avg(const double *M, const double *X, int64_t xs, int nb, double *Y, int64_t ys, int64_t n,
                      void *stream);
// H[f] = cu_f * mean_b dots[f*nb + b]  (per-frame covariance, MATLAB averaging)
int launch_fc_finish(const SolveArgs &a, const double *dots, double *H, int64_t hs, void *stream);
int launch_synth(const State *st, const SynthArgs &a, void *stream);
// WCE_MMSE_COV low-rank path: H (or, split, H_b per (frame, block) row) from
// the Gram system embedded at block row k0 (State::cov_k0)
// (rank = State::cov_rank: ranks 1..LRL_RMAX run one frame per lane instead)
// ranks 17..32, taps 0..r-1: 16 lanes per unit, two rows each (wce_lr_quad2.hip)
int launch_lr_quad2(const State *st, int rank, const SolveArgs &a, void *stream, int form = 0);
int launch_mmse_lr(const State *st, int k0, int rank, int taps, const SolveArgs &a, void *stream);
// the kernel launch_mmse_lr runs for `units` (frame, block) units (wce_debug_lr_kernel)
const char *lr_kernel_name(int k0, int rank, int taps, int64_t units);
// REF + WCE_MMSE_FRAME_COV (C semantics) in one launch: LT_LS of rx_pre, w at the
// pilots from State::Wp, s, u = Mu h and H = u s to a.w
int launch_ref_fc(const State *st, const SolveArgs &a, const double *rx_pre, int64_t ps, const double *tx_pre,
                  void *stream);
// TEXTBOOK per-frame covariance, C semantics: LT_LS of each preamble and u = Mu h in one launch (u rows at U, stride us)
int launch_fc_u(const State *st, const double *rx_pre, int64_t ps, const double *tx_pre, double *U, int64_t us,
                int64_t n, void *stream);
// the same w as full rows W[f] (zero off the pilots) from h rows X[f] (the variant path)
int launch_ref_w(const State *st, const double *X, int64_t xs, double *W, int64_t ws, int64_t n, void *stream);
// H[f] = mean of X rows 4f .. 4f+3 (MATLAB block average, left to right)
int launch_avg_blocks(const double *X, int64_t xs, double *H, int64_t hs, int64_t n, void *stream);
int set_flat_chunk(int64_t frames);   // wce_debug_set_flat_chunk
// kernel variants for A/B timing (wce_debug_set_variant)
constexpr int WCE_VARIANT_REF = 0;    // REF PS_MMSE: 0 = by batch size (default: one element per thread,
                                      // mmse_ref_elem_kernel, past REF_ELEM_FROM frames, else 512-element
                                      // chunks on a capped grid, mmse_ref_flat_kernel), 1 = always the capped
                                      // chunks, 2 = the chunks on an uncapped grid, 3 = always one element per
                                      // thread; bit-identical
constexpr int WCE_VARIANT_LS = 1;     // configs[1] LS: 2 = one element per thread (ls_elem_kernel, default),
                                      // 3 = the per-frame LIGHT ls_kernel
constexpr int WCE_VARIANT_REF_LS = 2;  // REF PS_MMSE + LS family (+ eq), C semantics: 0 = ref_ls_elem_kernel
                                      // (one element per thread, default), 1 = mmse_solve_ls_kernel (wave per frame)
constexpr int WCE_VARIANT_LR = 3;     // WCE_MMSE_COV low-rank path: 0 = ranks 1..LRL_RMAX one frame per lane
                                      // (mmse_lr_lane_kernel, direct or LDS-staged by batch size), ranks 9..16
                                      // 16 lanes per frame (mmse_lr_quad_kernel); default
                                      // 1 = every rank on mmse_lr_kernel (one frame per wave), 2 = lane kernel
                                      // direct, 3 / 4 = lane kernel staged, ranks 7-8 in the one- / two-
                                      // workgroups-per-CU build at any size; the lane and wave kernels agree
                                      // to rounding (~1e-15), not bitwise; the staged builds bitwise.
                                      // A diagonal Rhh runs the wave kernel's tap-domain Gram
                                      // (mmse_lr_kernel<K0, true>); 5 = the product Gram there instead
constexpr int WCE_VARIANT_REF_FC = 4;  // WCE_MMSE_FRAME_COV, C semantics: 0 = ref_fc_kernel (REF: LT_LS, the
                                      // u / w products and the read-out in one launch; TEXTBOOK: LT_LS and
                                      // u = Mu h in one launch; default), 1 = the LT_LS pass + the matvec
                                      // launches (+ the REF read-out); bit-identical
constexpr int WCE_VARIANT_COUNT = 5;
int variant_value(int which);
int set_variant(int which, int value);
int launch_ldc_convert(const void *src, void *dst, int64_t n, bool to_complex, void *stream);
int launch_nonfinite_scan(const double *H, int64_t stride, int64_t n, bool f32, uint32_t *bits,
                          unsigned long long *n_bad, void *stream);

// per-stream (or per-plan) scratch of wce_estimate: [frames] x 5 arrays of
// 64 complex (wce_api.cpp WS_ARRAYS / WS_LD); mu serialises the calls of one stream
struct Workspace {
    std::mutex mu;
    double *p = nullptr;
    int64_t frames = 0;
};

// wce_api.cpp hooks used by wce_multi.cpp: set wce_last_error() and return
// `code`; a context's device and whether its state is valid.
int api_fail(int code, const char *what);
int ctx_device(const wce_ctx *c);
bool ctx_ready(const wce_ctx *c);

}  // namespace wce
