/* wce_debug.h -- host-only hooks of libwce.so used by the parity tests to
 * check the 80-bit shared-state precompute without a GPU. */
#ifndef WCE_DEBUG_H
#define WCE_DEBUG_H
#ifdef __cplusplus
extern "C" {
#endif
/* F and the reference's cofactor invF (utils.c:141-170), 53*53 {re, im} long double pairs */
int wce_debug_reference_F(long double *out);
int wce_debug_reference_invF(long double *out);
/* the State wce_ctx_create builds: C (53*53 {re,im}), H_LT (53), sinc table (4*53), {a, b}, X mask */
int wce_debug_build_state(const double *tx_pre, const double *rx_pre, double ow2, int mode, double *C,
                          double *h_lt, double *sinc, double *ab, unsigned long long *xmask);
/* WCE_MMSE_COV state blob (wce_state_build_cov): the low-rank factor U
 * (C = U U^H; 53 rows x 64 columns {re, im}, zero past the rank), the rank,
 * the solve form (-1 dense, else the Gram system's first block row) and the
 * largest / smallest kept eigenvalue of C.  Outputs may be NULL. */
int wce_debug_cov_factor(const void *blob, size_t bytes, double *U, int *rank, int *k0, double *lmax, double *lmin);
/* A/B switch for the config-5 fusion (LS family + equalization in the MMSE
 * solve's epilogue); on by default.  ctx is a wce_ctx* (include/wce.h). */
struct wce_ctx;
int wce_debug_set_fusion(struct wce_ctx *ctx, int on);
/* A/B switch for the rank-1 path (TEXTBOOK / REF / FRAME_COV): a second
 * bordered row replaces the back-substitution and the C W product; on by
 * default.  Off: back-substitution + MFMA apply (shared modes). */
int wce_debug_set_border_dot(struct wce_ctx *ctx, int on);
/* Frames per launch of the flat-index kernels (LT_LS + PS_Linear, REF
 * PS_MMSE, the non-finite scan): 2^26 by default, so that 53 * frames < 2^32;
 * a smaller multiple of 32 makes tests reach the multi-launch path at small
 * sizes.  0 restores the default.  Process-wide. */
int wce_debug_set_flat_chunk(long long frames);
/* Kernel variant knobs for interleaved A/B timing and the gate's cross-checks
 * in one process (same buffers, same placement).  which 0: REF PS_MMSE (0 =
 * by batch size, default: one element per thread, mmse_ref_elem_kernel, past
 * 196,608 frames, else 512-element chunks on a capped grid; 1 = always the
 * capped chunks; 2 = the chunks on an uncapped grid; 3 = always one element
 * per thread).
 * which 1: LT_LS + PS_Linear in C semantics (2 = one element per thread,
 * ls_elem_kernel, default; 3 = the per-frame LIGHT kernel).  which 2: REF
 * PS_MMSE with LS outputs in one call (0 = one element per thread,
 * ref_ls_elem_kernel, default; 1 = the wave-per-frame fused solve).
 * which 3: WCE_MMSE_COV low-rank path (0 = ranks 1..8 one frame per lane in
 * the LDS-staged form, mmse_lr_lane_staged_kernel, ranks 7 and 8 in its
 * two-workgroups-per-CU build past 65,536 units on a 256-CU device, and
 * ranks 9..16 16 lanes per frame, mmse_lr_quad_kernel, default; 1 = every
 * rank one frame per wave; 2 = the lane kernel's direct form,
 * mmse_lr_lane_kernel; 3 / 4 = the staged form with ranks 7 and 8 in the
 * one- / two-workgroups-per-CU build at any size; 2..4: ranks past 8 one
 * frame per wave).  which 4: REF + WCE_MMSE_FRAME_COV in C semantics (0 =
 * ref_fc_kernel, one launch, default; 1 = the LT_LS pass, two matvec
 * launches and the REF read-out).
 * Process-wide; the variants of which 0, 1, 2, 4 give bit-identical results,
 * which 3's kernels sum in different orders and agree to rounding (tests
 * check both).  (Round 4 retired ls_flat_kernel -- which 1 = 0, 1 -- and the
 * REF frame tiles -- which 0 = 1.) */
int wce_debug_set_variant(int which, int value);
/* WCE_MMSE_COV solve form for A/B and accuracy probes: 0 = as the state
 * chose (default), 1 = always the dense Ryy solve, 2 = always the low-rank
 * Gram path (at the state's rank).  ctx is a wce_ctx*. */
int wce_debug_set_cov_path(struct wce_ctx *ctx, int path);
/* The kernel a WCE_MMSE_COV low-rank estimate over `units` (frame, block)
 * units runs under the current variant (e.g. "mmse_lr_lane_staged_kernel<8, 2>");
 * "" for a ctx on the dense path.  For bench labels and the gate's checks. */
const char *wce_debug_lr_kernel(struct wce_ctx *ctx, long long units);
/* A/B switch of the constant-modulus path (wce_ctx_set_modulus); on by default. */
int wce_debug_set_cm(struct wce_ctx *ctx, int on);
/* How many times the compat WiFi_channel_estimation_PS_MMSE built and
 * uploaded its shared state (main.c:148's F / H_EST_LS / ow2): once per
 * distinct (F, H_EST_LS, ow2), not once per call.  0 before the first call. */
unsigned long long wce_debug_compat_state_builds(void);
#ifdef __cplusplus
}
#endif
#endif
