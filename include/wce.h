/*
 * wce.h -- C ABI of the MI355X 802.11 channel-estimation engine (libwce.so).
 *
 * Drop-in boundary for the estimator path of usmandroid/80211ParallelEstimation
 * (main.c / utils.c).  Plain pointers and sizes only: no HIP or torch types in
 * the signatures (streams are passed as `void *` hipStream_t, NULL = default
 * stream).  Every call returns an int status (0 ok, < 0 error); the reference
 * functions return void and print on dimension mismatch (utils.c:18-19).
 *
 * Two layers:
 *   1. the batched API below (wce_ctx_*, wce_estimate, wce_mmse_*) that runs
 *      B frames resident in HBM through hand-written gfx950 kernels;
 *   2. include/wce_compat.h: the five reference signatures of main.c:4-8,
 *      one frame in host memory, implemented on top of layer 1.
 *
 * Data layout: complex fp64 is {re, im} (16 B, binary-compatible with C99
 * double _Complex and hipDoubleComplex).  Frame f, OFDM block b, subcarrier k
 * lives at base[f*frame_stride + b*block_stride + k] (strides in elements);
 * the reference's block-major inputs.h layout (tx_symb[53*15]) is
 * frame_stride = 795, block_stride = 53.
 */
#ifndef WCE_H
#define WCE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define WCE_NSC 53   /* SAMPUTIL, utils.h:13 */
#define WCE_NBLK 15  /* OFDMBLK,  utils.h:15 */
#define WCE_DC 26    /* main.c:74 H_EST[26] = 0 */
#define WCE_P0 5     /* utils.h:16-19 pilot subcarriers */
#define WCE_P1 19
#define WCE_P2 33
#define WCE_P3 47

typedef struct { double re, im; } wce_complex;

enum {
    WCE_OK = 0,
    WCE_EINVAL = -1,   /* bad argument / shape */
    WCE_EHIP = -2,     /* HIP runtime error */
    WCE_ENOMEM = -3,
    WCE_ESTATE = -4,   /* context has no valid shared state */
    WCE_ENODEV = -5    /* no usable gfx950 device */
};

/* estimator mask bits (one per reference entry point, main.c:4-8) */
#define WCE_EST_LT_LS     (1u << 0)  /* WiFi_channel_estimation_LT_LS     main.c:66  */
#define WCE_EST_PS_LINEAR (1u << 1)  /* WiFi_channel_estimation_PS_Linear main.c:77  */
#define WCE_EST_PS_CUBIC  (1u << 2)  /* WiFi_channel_estimation_PS_Cubic  main.c:103 */
#define WCE_EST_PS_SINC   (1u << 3)  /* WiFi_channel_estimation_PS_Sinc   main.c:124 */
#define WCE_EST_PS_MMSE   (1u << 4)  /* WiFi_channel_estimation_PS_MMSE   main.c:148 */
#define WCE_EQUALIZE      (1u << 5)  /* WiFi_Equalization.m (no C original) */
#define WCE_EST_LS_ALL    (0xFu)
/* PS_MMSE with each frame's own covariance: Rhh_f from the frame's preamble
 * (wce_frames.rx_pre required) instead of the context's shared preamble, i.e.
 * main.c's PS_MMSE called with H_EST_LS = that frame's LT_LS (main.c:41-53 per
 * frame).  C_f = F Rhh_f F^H is rank 1, so it is never formed: two batched
 * MFMA matrix-vector products give its factors and the solve writes H. */
#define WCE_MMSE_FRAME_COV (1u << 6)

/* MMSE semantics (DESIGN.md "MMSE contract"):
 *  REF      : main.c:148-212 with the NaN inverse(Ryy) repaired:
 *             H = C_ref X4 (2 ow2 I)^-1 rx, C_ref = F Rhh FH, X4 = pilots of tx.
 *  TEXTBOOK : WiFi_channel_estimation_PS_MMSE.m per block:
 *             H = C X (X C X' + ow2 I)^-1 rx, C = F Rhh F', X = diag(tx).
 * Both run the same kernel: H = C X (a X C X' + b I)^-1 rx. */
enum { WCE_MMSE_REF = 0, WCE_MMSE_TEXTBOOK = 1, WCE_MMSE_COV = 2 };
/*  COV      : TEXTBOOK with a caller-supplied channel covariance Rhh instead
 *             of the single-preamble estimate ifft(H_LT) ifft(H_LT)' (e.g. a
 *             power-delay-profile model or an average over many preambles):
 *             C = F Rhh F', generally full rank -- the dense per-frame solve
 *             is then the only way to apply it.  See wce_state_build_cov. */

typedef struct wce_ctx wce_ctx;

/* Build the shared state on the host (F as main.c:18-26 builds it, the
 * reference's cofactor invF of utils.c:141-170 in 80-bit long double, H_LT
 * from the shared preamble (main.c:66-75), the MMSE covariance C of
 * main.c:186-203, the sinc table of utils.c:727-733) and upload it to `device`.  tx_pre/rx_pre: the shared
 * preamble FFTs (53 each, host).  The first call in a process spends
 * ~0.5 s (8 threads) on invF; later calls reuse it. */
int wce_ctx_create(wce_ctx **ctx, int device, const wce_complex *tx_pre,
                   const wce_complex *rx_pre, double ow2, int mmse_mode);

/* A context whose device state is filled later (e.g. by an RCCL broadcast
 * into the buffer returned by wce_ctx_state). */
int wce_ctx_create_empty(wce_ctx **ctx, int device);
int wce_ctx_destroy(wce_ctx *ctx);

/* WCE_MMSE_COV: Rhh is the 53 x 53 time-domain channel covariance (row-major,
 * Hermitian positive semidefinite, host); tx_pre/rx_pre still give H_LT for
 * LT_LS and equalization.  Rhh is checked: WCE_EINVAL unless every entry is
 * finite, Rhh = Rhh^H to 1e-12 of its largest entry, and its eigenvalues are
 * >= -1e-12 of the largest.  The 80-bit eigendecomposition Rhh = V Lambda V^H
 * (eigenvalues at or below 2^-46 of the largest -- the rounding level of an
 * fp64 input -- count as zero) gives C = F Rhh F^H = U U^H, U = F V sqrt(Lambda),
 * r columns.  The per-frame solve then runs in one of two forms:
 *   low rank (r < 53, or a spectrum wider than 1e5): the r x r Gram system
 *     (a G^H G + b I) t = G^H rx, G = X U, and H = U s -- accurate to ~1e-13
 *     at any rank (the dense form loses ~eps cond(Ryy) there);
 *   dense (r = 53 and a spectrum within 1e5): Cholesky of Ryy, then H = C W on MFMA. */
int wce_ctx_create_cov(wce_ctx **ctx, int device, const wce_complex *tx_pre, const wce_complex *rx_pre,
                       const wce_complex *Rhh, double ow2);
/* WCE_MMSE_COV context: the rank r, whether the low-rank path runs (1) or the
 * dense one (0), and the largest / smallest kept eigenvalue of C (outputs may be NULL). */
int wce_ctx_cov_info(wce_ctx *ctx, int *rank, int *low_rank, double *lambda_max, double *lambda_min);
/* WCE_MMSE_COV, constant-modulus frames (round 4; WiFi_channel_estimation_PS_MMSE.m:29-32).
 * Ryy depends on a frame's symbols only through P = diag |x_k|^2 (and their
 * phases), and for PSK frames -- the reference's BPSK data (inputs.h), QPSK --
 * P is the same for every frame.  x_ref: one frame's 53 symbols; p_k = |x_ref,k|^2
 * (0 off the X mask) is the pattern.  The ctx forms once, in 80-bit on the
 * host, K = (a C P + b I)^-1 C (the push-through of C X^H Ryy^-1) and uploads
 * it.  Estimates in C semantics then check every frame on the device: a frame
 * whose |x_k|^2 equals p_k bit for bit on all subcarriers takes
 *     H = K (conj(x) o rx)   [+ C ((x - conj x) o (rx - a x o H1)) / b for non-real x]
 * -- two batched f64-MFMA products, no per-frame factorisation -- and every
 * other frame the per-frame solve, as without the pattern.  Ranks <= 8 keep
 * the one-frame-per-lane kernels (already bound by the frames' HBM traffic).
 * x_ref NULL: off.  Needs the ctx that built the state (wce_ctx_create_cov);
 * it updates the shared state, so a multi-GPU run sets it before the
 * broadcast.  Not safe against estimates in flight on this ctx. */
int wce_ctx_set_modulus(wce_ctx *ctx, const wce_complex *x_ref);

/* Device pointer and size of the packed shared state (C, H_LT, tx_pre, sinc
 * table, MMSE coefficients): the single buffer a multi-GPU run broadcasts
 * from rank 0.  After writing it externally call wce_ctx_mark_ready. */
int wce_ctx_state(wce_ctx *ctx, void **device_ptr, size_t *bytes);
int wce_ctx_mark_ready(wce_ctx *ctx);

/* Host-only shared state: build it once (no device needed), ship the bytes
 * to other processes / devices (RCCL broadcast, file, ...), and load them
 * into a context.  wce_state_size() is the byte size of that blob. */
size_t wce_state_size(void);
int wce_state_build(void *host_state, size_t bytes, const wce_complex *tx_pre, const wce_complex *rx_pre,
                    double ow2, int mmse_mode);
int wce_state_build_cov(void *host_state, size_t bytes, const wce_complex *tx_pre, const wce_complex *rx_pre,
                        const wce_complex *Rhh, double ow2);
int wce_ctx_load_state(wce_ctx *ctx, const void *host_state, size_t bytes);
/* wce_ctx_set_modulus on a host blob built by wce_state_build_cov from the same Rhh. */
int wce_state_set_modulus(void *host_state, size_t bytes, const wce_complex *Rhh, const wce_complex *x_ref);
/* Host-only check of a state blob (e.g. bytes received from another rank):
 * WCE_OK and its MMSE mode (may be NULL) if it holds a valid state, else
 * WCE_EINVAL (too short) / WCE_ESTATE (no valid magic). */
int wce_state_validate(const void *host_state, size_t bytes, int *mmse_mode);

/* Copy back the shared vectors (host outputs, may be NULL): H_LT (53),
 * C (53*53 row-major), and the MMSE coefficients a, b. */
int wce_ctx_get_shared(wce_ctx *ctx, wce_complex *h_lt, wce_complex *C, double *a, double *b);

typedef struct {
    const wce_complex *tx;      /* device; tx[f*frame_stride + b*block_stride + k] */
    const wce_complex *rx;      /* device; same layout as tx */
    const wce_complex *rx_pre;  /* device; per-frame preamble FFT rx_pre[f*pre_stride + k],
                                   NULL = use the context's shared H_LT */
    const wce_complex *tx_pre;  /* device; shared preamble (53), NULL = context's */
    int64_t frame_stride;
    int64_t block_stride;
    int64_t pre_stride;
    int64_t n_frames;
    int32_t block;              /* OFDM block read by PS_* / MMSE (main.c:16 uses 0) */
    int32_t semantics;          /* WCE_SEM_C (main.c) or WCE_SEM_MATLAB (WiFi_*.m) */
} wce_frames;

/* Estimator semantics (wce_frames.semantics):
 *  WCE_SEM_C      : main.c -- one OFDM block (`block`), LT_LS "conj" quirk
 *                   (main.c:69), every cubic divided difference by 14 (main.c:116-118).
 *  WCE_SEM_MATLAB : WiFi_channel_estimation_*.m -- proper conj in LT_LS, PS_* and
 *                   PS_MMSE averaged over OFDM blocks 1..4 (0..3 here; `block`
 *                   ignored), cubic divisors 14/28/42 (PS_Cubic.m:11-13). */
enum { WCE_SEM_C = 0, WCE_SEM_MATLAB = 1 };

typedef struct {
    wce_complex *lt_ls;         /* device [n_frames][out_stride], NULL = not requested */
    wce_complex *ps_linear;
    wce_complex *ps_cubic;
    wce_complex *ps_sinc;
    wce_complex *ps_mmse;
    wce_complex *eq;            /* equalized symbols, eq[f*eq_frame_stride + b*eq_block_stride + k] */
    int64_t out_stride;         /* >= 53 */
    int64_t eq_frame_stride;
    int64_t eq_block_stride;
    uint32_t eq_source;         /* PS estimate blended with H_LT (WiFi_RX.m:60 uses PS_Linear);
                                   0 = WCE_EST_PS_LINEAR */
    uint32_t flags;             /* WCE_OUT_* */
} wce_outputs;

/* wce_outputs.flags.  WCE_OUT_LS_F32: the LS family (lt_ls, ps_linear,
 * ps_cubic, ps_sinc) and eq are stored as complex float ({re, im} float, 8 B),
 * computed in fp64 and rounded once (BASELINE configs[4] "mixed fp64 solve /
 * fp32 interp"; <= 1e-7 relative).  ps_mmse stays complex double.  Strides
 * count elements of each buffer's own type. */
#define WCE_OUT_LS_F32 (1u << 0)

/* Threading: one ctx may serve calls on several streams at once, from one
 * host thread or several.  The shared state is read-only after creation, and
 * the scratch that WCE_MMSE_FRAME_COV and MATLAB-semantics PS_MMSE need
 * (5 KB per frame) is kept per stream, so calls on different streams never
 * share it; calls on the same stream are serialised (as the stream would).
 * Plans own their scratch.  wce_last_error() is per thread.
 *
 * Pre-size that scratch for batches of up to n_frames so that wce_estimate
 * never allocates: _stream for one stream; wce_ctx_reserve for the NULL
 * stream, and as the minimum size of every stream's scratch created later.
 * Without it the first larger batch on a stream allocates (synchronously on
 * that stream) and keeps the buffer until wce_ctx_destroy. */
int wce_ctx_reserve(wce_ctx *ctx, int64_t n_frames);
int wce_ctx_reserve_stream(wce_ctx *ctx, int64_t n_frames, void *stream);

/* Run the estimators selected in `mask` over all frames, asynchronously on
 * `stream`.  Replaces the per-frame calls of main.c:37-54 (and the frame
 * loops of main_openmp.c / main_mpi.c) with one batched call.  LS family + equalization: one HBM-streaming kernel; MMSE: the
 * LDS/register-resident Cholesky solve kernel followed by the MFMA GEMM
 * (the ps_mmse buffer doubles as the solve->GEMM workspace). */
int wce_estimate(wce_ctx *ctx, const wce_frames *in, const wce_outputs *out,
                 uint32_t mask, void *stream);

/* Launch plans: one wce_estimate call (fixed buffers, strides, mask, batch)
 * captured into a HIP graph once and replayed with a single graph launch --
 * for serving loops that re-run small batches into the same buffers, where
 * per-call host checks and kernel launch latency dominate.  Arguments are
 * validated and the plan's own workspace sized at creation; the plan keeps
 * raw pointers, so the buffers and the ctx (its device state) must outlive
 * it.  Capture runs on a private stream; launches go to the stream given, and
 * replays may run beside direct calls on other streams.  A replay is one
 * graph launch; on ROCm 7 that measured slightly SLOWER than the direct
 * call's launches (bench small_batch), so a plan buys validation once and a
 * fixed argument set, not speed. */
typedef struct wce_plan wce_plan;
int wce_plan_create(wce_plan **plan, wce_ctx *ctx, const wce_frames *in, const wce_outputs *out,
                    uint32_t mask);
int wce_plan_launch(wce_plan *plan, void *stream);
int wce_plan_destroy(wce_plan *plan);

/* The two MMSE stages, exposed for profiling:
 *   solve: W[f] = X_f (a X_f C X_f' + b I)^-1 rx_f        (FP64 VALU, per frame)
 *   apply: H[f] = C W[f]                                  (FP64 MFMA batched GEMM)
 * W and H may alias (in place). */
int wce_mmse_solve(wce_ctx *ctx, const wce_frames *in, wce_complex *W, int64_t w_stride, void *stream);
int wce_mmse_apply(wce_ctx *ctx, const wce_complex *W, wce_complex *H, int64_t stride,
                   int64_t n_frames, void *stream);

/* Synthetic 802.11 frames generated on the device from a counter-based RNG
 * keyed by (seed, global frame index), so any shard regenerates identical
 * frames: BPSK data +-A, pilots A*(1,1,1,-1)*p_b (802.11 polarity), DC = 0,
 * a 6-tap exponential-PDP channel (or h_shared for every frame, if non-NULL),
 * CN(0, ow2) noise.  rx_pre (may be NULL) = per-frame preamble H*tx_pre + noise/sqrt2. */
int wce_synth_frames(wce_ctx *ctx, wce_complex *tx, wce_complex *rx, wce_complex *rx_pre,
                     int64_t frame_stride, int64_t block_stride, int64_t pre_stride,
                     int64_t first_frame, int64_t n_frames, uint64_t seed,
                     const wce_complex *h_shared, double amplitude, double ow2, void *stream);

/* ---- time-domain front end (MATLAB only, no C original) ----
 * WiFi_blocks_extraction.m:1-11: OFDM block b of frame f is the 80 samples
 * samples[f*packet_stride + 80 b + (0..79)]; the 16-sample cyclic prefix is
 * dropped and the last 64 go through a 64-point DFT, circshift(., 26), and
 * the first 53 bins are kept:
 *     sym[f*frame_stride + b*block_stride + i] = DFT64[(i - 26) mod 64],  i < 53.
 * Used for tx and rx packets alike (WiFi_RX.m:42-43).  The output is the
 * wce_frames layout, so wce_estimate can consume it directly.  The ctx only
 * selects the device (its state need not be loaded). */
enum { WCE_FFT_SIZE = 64, WCE_SAMPLES_PER_BLOCK = 80 };
int wce_front_end_blocks(wce_ctx *ctx, const wce_complex *samples, int64_t packet_stride, int64_t n_frames,
                         int32_t n_blocks, wce_complex *sym, int64_t frame_stride, int64_t block_stride,
                         void *stream);

/* WiFi_RX.m:18-30: the long training field of frame f is
 * lptot[f*lptot_stride + (0..lptot_len-1)]; its last 64 samples are p1 and
 * the 64 before them p2.  pre_fft[f*pre_stride + i] = circshift(DFT64((p1+p2)/2), 26)[i],
 * i < 53 (feed it to wce_frames.rx_pre / tx_pre), and, if ow2 != NULL,
 * ow2[f] = sum |p2 - p1|^2 / (2*64), the noise estimate of WiFi_RX.m:30. */
int wce_front_end_preamble(wce_ctx *ctx, const wce_complex *lptot, int64_t lptot_stride, int64_t lptot_len,
                           int64_t n_frames, wce_complex *pre_fft, int64_t pre_stride, double *ow2,
                           void *stream);

/* Non-finite guard.  The reference passes NaN/Inf through
 * silently: main.c's PS_MMSE returns NaN x 53 (main.c:148-212), a zero pilot
 * makes PS_* divide by zero (main.c:82-84), and its dimension checks only
 * print (utils.c:18-19).  One HBM pass over an output array H[f*stride + k]
 * (k < 53; complex double, or complex float with flags = WCE_OUT_LS_F32):
 * bit f % 32 of bitmap[f / 32] (device, ceil(n/32) words, zeroed here) is set
 * iff any of frame f's 53 entries has a NaN or Inf part; *n_bad (device,
 * optional) receives the number of such frames.  Any ctx selects the device
 * (its state need not be loaded).  Asynchronous on `stream`. */
int wce_nonfinite_scan(wce_ctx *ctx, const void *H, int64_t stride, int64_t n_frames, uint32_t flags,
                       uint32_t *bitmap, unsigned long long *n_bad, void *stream);

/* The reference's data format on the device.  Its arrays are `long double
 * complex` (main.c:4-8): on x86-64, two x87 80-bit extended values in 16-byte
 * slots (32 B per complex; bytes 10-15 of a slot are padding).  A host that
 * keeps frames in that format copies the raw bytes to the device and converts
 * there:
 *   wce_ldc_to_complex: n complex values, x87 -> fp64, rounded exactly as the
 *     C cast (double)x on x86 (nearest-even, overflow to Inf, gradual
 *     underflow; NaNs quieted and truncated; invalid encodings -> the x87
 *     default NaN);
 *   wce_complex_to_ldc: fp64 -> x87, exact (the C cast (long double)x),
 *     padding written as zero.
 * Device pointers, 16-byte aligned, not overlapping; asynchronous on
 * `stream` (current device). */
int wce_ldc_to_complex(const void *src, wce_complex *dst, int64_t n, void *stream);
int wce_complex_to_ldc(const wce_complex *src, void *dst, int64_t n, void *stream);

/* ---- multi-GPU: frames are independent, so a batch is sharded
 * over GPUs with no data-path collective; the only exchange is ONE RCCL
 * broadcast of the packed shared state (wce_ctx_state) over xGMI, the
 * analogue of the reference's MPI_Bcast of F / Ryy (main_mpi.c:687-688,
 * 727-728).  RCCL (librccl.so.1) is loaded on first use, so hosts that never
 * call these need no RCCL.  Two launch models:
 *   - one process per GPU (the MPI model of main_mpi.c): rank 0 calls
 *     wce_comm_unique_id, the host distributes the WCE_COMM_ID_BYTES bytes
 *     (MPI_Bcast, a file, a socket), every rank calls wce_comm_init_rank;
 *   - one process driving several GPUs: wce_comm_init_all. */
#define WCE_COMM_ID_BYTES 128
typedef struct wce_comm wce_comm;
int wce_comm_unique_id(void *id);
int wce_comm_init_rank(wce_comm **comm, const void *id, int nranks, int rank, int device);
int wce_comm_init_all(wce_comm **comms, int ndev, const int *devices);
int wce_comm_destroy(wce_comm *comm);
int wce_comm_info(const wce_comm *comm, int *rank, int *nranks, int *device);

/* ONE in-place ncclBroadcast of ctx's shared state from `root` (whose ctx
 * must hold a valid state) into every rank's ctx (which may be empty, see
 * wce_ctx_create_empty); ctx and comm must be on the same device.  Returns
 * once the state has arrived and been validated (a once-per-process setup
 * call, not a per-batch one).  The _all form does the same for n contexts of
 * one process (comms from wce_comm_init_all), as one RCCL group. */
int wce_ctx_broadcast_state(wce_ctx *ctx, wce_comm *comm, int root, void *stream);
int wce_ctx_broadcast_state_all(wce_ctx **ctxs, wce_comm **comms, int n, int root, void **streams);

/* max over ranks of one double (e.g. each shard's parity error, or its time):
 * an 8-byte ncclAllReduce, synchronous.  _all: one value per context of one
 * process, every entry replaced by the maximum. */
int wce_comm_max_f64(wce_comm *comm, double *value, void *stream);
int wce_comm_max_f64_all(wce_comm **comms, int n, double *values, void **streams);

/* Contiguous frame range [first, first + count) of `rank` out of `total`
 * (the first total % nranks ranks take one extra frame). */
int wce_shard(int64_t total, int nranks, int rank, int64_t *first, int64_t *count);

/* ---- thin runtime helpers (so C hosts and tests need no other HIP binding) ---- */
int wce_device_count(int *count);
int wce_set_device(int device);
int wce_malloc(void **ptr, size_t bytes);
int wce_free(void *ptr);
int wce_memcpy_htod(void *dst, const void *src, size_t bytes);
int wce_memcpy_dtoh(void *dst, const void *src, size_t bytes);
int wce_memcpy_dtod(void *dst, const void *src, size_t bytes, void *stream);
int wce_memset(void *dst, int value, size_t bytes);
/* pinned (page-locked) host memory and stream-ordered copies, for hosts that
 * keep frames in host memory and overlap PCIe transfers with estimation */
int wce_host_alloc(void **ptr, size_t bytes);
int wce_host_free(void *ptr);
int wce_memcpy_htod_async(void *dst, const void *src, size_t bytes, void *stream);
int wce_memcpy_dtoh_async(void *dst, const void *src, size_t bytes, void *stream);
int wce_stream_create(void **stream);
int wce_stream_destroy(void *stream);
int wce_stream_synchronize(void *stream);
int wce_event_create(void **event);
int wce_event_destroy(void *event);
int wce_event_record(void *event, void *stream);
int wce_event_elapsed_ms(float *ms, void *start, void *stop);
const char *wce_last_error(void);
const char *wce_version(void);

#ifdef __cplusplus
}
#endif
#endif /* WCE_H */
