/*
 * wce_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference's 802.11 channel-estimation path
 * (usmandroid/80211ParallelEstimation, main.c / utils.c), used as the parity
 * checker for the MI355X engine.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library.  The product
 * (80211parallelestimation_amd/, libwce.so) never links or calls it.
 *
 * Parity pinning (see DESIGN.md "Oracle"):
 *   - LS family, invF and the REF-repaired MMSE are checked bit-for-bit
 *     against the reference's own functions compiled from /root/reference
 *     (oracle/_ref, recipe in oracle/Makefile) -> tests/golden/ref_*.npz.
 *   - The per-block LS kernels and the equalizer are also pinned against
 *     the MATLAB workspace matlab.mat (tests/golden/matlab_pins.npz).
 *   - TEXTBOOK MMSE (WiFi_channel_estimation_PS_MMSE.m semantics) has no
 *     reference output; it is pinned only against its closed form
 *     ("parity unpinned" against the reference).
 *
 * Arithmetic: long double _Complex (x87 80-bit) exactly like the reference,
 * with the same operation order, so that gcc lowers the same __mulxc3 /
 * __divxc3 calls.  creal()/cimag() round through double where the reference
 * calls them (glibc's creal takes double _Complex).
 */
#include <complex.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>
#include <omp.h>

typedef long double complex ldc;

#define N 53            /* SAMPUTIL  utils.h:13 */
#define NBLK 15         /* OFDMBLK   utils.h:15 */
#define P0 5            /* utils.h:16-19 */
#define P1 19
#define P2 33
#define P3 47
#define DC 26

/* main.c:18-26: F[t][f] = cexp(-2*I*PI*t*f/SAMPUTIL).  I is float _Complex,
 * so the argument is formed and evaluated in double. */
void orc_fmatrix(ldc *F)
{
    for (int f = 0; f < N; f++)
        for (int t = 0; t < N; t++)
            F[t * N + f] = cexp(-2 * I * M_PI * t * f / N);
}

/* main.c:66-75.  conj = creal(tx) - cimag(tx) is a REAL value (quirk), so
 * H = (c*rx)/(c*tx).  H[26] = 0. */
void orc_lt_ls(const ldc *tx_pre, const ldc *rx_pre, ldc *H)
{
    ldc conj1, conj2;
    for (int i = 0; i < 26; i++) {
        conj1 = creal(tx_pre[i]) - cimag(tx_pre[i]);
        conj2 = creal(tx_pre[i + 27]) - cimag(tx_pre[i + 27]);
        H[i] = (conj1 * rx_pre[i]) / (conj1 * tx_pre[i]);
        H[i + 27] = (conj2 * rx_pre[i + 27]) / (conj2 * tx_pre[i + 27]);
    }
    H[26] = 0.0;
}

static void pilot_ls(const ldc *tx, const ldc *rx, ldc hp[4])
{
    const int P[4] = {P0, P1, P2, P3};
    for (int i = 0; i < 4; i++) hp[i] = rx[P[i]] / tx[P[i]];
}

/* main.c:77-101.  Three linear segments; k>=P3 extrapolates segment 2
 * (main.c:96-98), k<P0 extrapolates segment 0. */
void orc_ps_linear(const ldc *tx, const ldc *rx, ldc *H)
{
    ldc hp[4];
    long double alpha, delta = P1 - P0;
    pilot_ls(tx, rx, hp);
    for (int i = 0; i < N; i++) {
        if (i < P1) {
            alpha = (i - P0) / delta;
            H[i] = hp[0] + ((hp[1] - hp[0]) * alpha);
        } else if (i < P2) {
            alpha = (i - P1) / delta;
            H[i] = hp[1] + ((hp[2] - hp[1]) * alpha);
        } else {                       /* P2 <= i < P3 and i >= P3 share a segment */
            alpha = (i - P2) / delta;
            H[i] = hp[2] + ((hp[3] - hp[2]) * alpha);
        }
    }
}

/* main.c:103-122.  Newton form; every divided difference divides by
 * delta = 14 (quirk; MATLAB divides by 14, 28, 42). */
void orc_ps_cubic(const ldc *tx, const ldc *rx, ldc *H)
{
    ldc hp[4], f0, f01, f12, f23, f012, f123, f0123;
    long double delta = P1 - P0;
    pilot_ls(tx, rx, hp);
    f0 = hp[0];
    f01 = (hp[1] - hp[0]) / delta;
    f12 = (hp[2] - hp[1]) / delta;
    f23 = (hp[3] - hp[2]) / delta;
    f012 = (f12 - f01) / delta;
    f123 = (f23 - f12) / delta;
    f0123 = (f123 - f012) / delta;
    for (int k = 0; k < N; k++)
        H[k] = f0 + f01 * (k - P0) + f012 * (k - P0) * (k - P1)
             + f0123 * (k - P0) * (k - P1) * (k - P2);
}

/* utils.c:727-733 */
static double ref_sinc(double x) { return x != 0 ? sin(M_PI * x) / (M_PI * x) : 1; }

/* main.c:124-146.  Pilot LS rounded to double complex; products and the
 * four-term sum in double. */
void orc_ps_sinc(const ldc *tx, const ldc *rx, ldc *H)
{
    double complex hp[4], s1, s2, s3, s4;
    long double delta = P1 - P0;
    const int P[4] = {P0, P1, P2, P3};
    double a, b, c, d;
    for (int i = 0; i < 4; i++) hp[i] = rx[P[i]] / tx[P[i]];
    for (int k = 0; k < N; k++) {
        a = (k - P0) / delta;
        b = (k - P1) / delta;
        c = (k - P2) / delta;
        d = (k - P3) / delta;
        s1 = hp[0] * ref_sinc(a);
        s2 = hp[1] * ref_sinc(b);
        s3 = hp[2] * ref_sinc(c);
        s4 = hp[3] * ref_sinc(d);
        H[k] = s1 + s2 + s3 + s4;
    }
}

/* ---------------- dense helpers (utils.c), row-major n x n ------------- */

/* utils.c:543-569: determinant by unpivoted Schur recursion
 * S[i-1][j-1] = m[i][j] - m[i][0]*m[0][j]/m[0][0]. */
static ldc det_rec(const ldc *m, int order, ldc *scratch)
{
    if (order == 1) return m[0];
    if (order == 2) return m[0] * m[3] - m[1] * m[2];
    int s = order - 1;
    ldc *sub = scratch;
    for (int i = 1; i < order; i++)
        for (int j = 1; j < order; j++)
            sub[(i - 1) * s + (j - 1)] = m[i * order + j] - (m[i * order] * m[j] / m[0]);
    return m[0] * det_rec(sub, s, scratch + (size_t)s * s);
}

static size_t det_scratch(int order)
{
    size_t t = 0;
    for (int s = order - 1; s >= 1; s--) t += (size_t)s * s;
    return t + 1;
}

/* utils.c:141-170 + GetMinor utils.c:440-459: adjugate inverse,
 * Y[i][j] = (1/det(A)) * det(minor(A, j, i)) * (-1)^(i+j).
 * Cofactors are independent, so they are spread over OpenMP threads; each
 * one uses the reference's exact operation order. */
void orc_inverse_cofactor(const ldc *A, int order, ldc *Y)
{
    ldc *scr0 = malloc(sizeof(ldc) * det_scratch(order));
    ldc det = 1.0 / det_rec(A, order, scr0);
    free(scr0);
    int m = order - 1;
#pragma omp parallel
    {
        ldc *minor = malloc(sizeof(ldc) * (size_t)m * m);
        ldc *scr = malloc(sizeof(ldc) * det_scratch(m));
#pragma omp for schedule(dynamic)
        for (int jj = 0; jj < order * order; jj++) {
            int j = jj / order, i = jj % order;
            int rc = 0;
            for (int r = 0; r < order; r++) {
                if (r == j) continue;
                int cc = 0;
                for (int c = 0; c < order; c++) {
                    if (c == i) continue;
                    minor[rc * m + cc] = A[r * order + c];
                    cc++;
                }
                rc++;
            }
            ldc v = det * det_rec(minor, m, scr);
            if ((i + j) % 2 == 1) v = (-1) * v;
            Y[i * order + j] = v;
        }
        free(minor);
        free(scr);
    }
}

/* utils.c:16-31: res = M1 (r1 x c1) * M2 (c1 x c2), sum = sum + a*b. */
static void mat_mul(const ldc *M1, int r1, int c1, const ldc *M2, int c2, ldc *res)
{
    for (int c = 0; c < r1; c++)
        for (int d = 0; d < c2; d++) {
            ldc sum = 0;
            for (int k = 0; k < c1; k++) sum = sum + M1[c * c1 + k] * M2[k * c2 + d];
            res[c * c2 + d] = sum;
        }
}

/* utils.c:3-7: "hermitian" = transpose of the REAL value creal - cimag. */
static void mat_hermitian_quirk(const ldc *M, int n, ldc *res)
{
    for (int r = 0; r < n; r++)
        for (int c = 0; c < n; c++)
            res[c * n + r] = creal(M[r * n + c]) - cimag(M[r * n + c]);
}

/*
 * REF-repaired PS_MMSE (main.c:148-212).  Same pipeline and operation order
 * as the reference with ONE deviation: inverse(Ryy) (main.c:201), which the
 * unpivoted cofactor routine turns into NaN, is replaced by the exact
 * inverse of the diagonal Ryy = 2*ow2*I (addition() returns M1+M1,
 * utils.c:117).  Dead stores main.c:194-196 are skipped (they do not reach
 * the output).  invF may be NULL (computed here, ~0.5 s with OpenMP).
 */
void orc_mmse_ref_repaired(const ldc *tx, const ldc *rx, const ldc *F, double ow2,
                           const ldc *H_LS, const ldc *invF_in, ldc *H)
{
    const int P[4] = {P0, P1, P2, P3};
    ldc *FH = calloc(N * N, sizeof(ldc)), *X4 = calloc(N * N, sizeof(ldc));
    ldc *Rhh = calloc(N * N, sizeof(ldc)), *Rhy = calloc(N * N, sizeof(ldc));
    ldc *invF = calloc(N * N, sizeof(ldc)), *t1 = calloc(N * N, sizeof(ldc));
    ldc *g = calloc(N, sizeof(ldc)), *q = calloc(N, sizeof(ldc));
    ldc *t3 = calloc(N, sizeof(ldc)), *invRyy = calloc(N * N, sizeof(ldc));
    for (int p = 0; p < 4; p++) X4[P[p] * N + P[p]] = tx[P[p]];       /* main.c:166-181 */
    mat_hermitian_quirk(F, N, FH);                                       /* main.c:183 */
    if (invF_in) memcpy(invF, invF_in, sizeof(ldc) * N * N);
    else orc_inverse_cofactor(F, N, invF);                               /* main.c:186 */
    mat_mul(invF, N, N, H_LS, 1, g);                                     /* main.c:187 */
    for (int c = 0; c < N; c++) q[c] = creal(g[c]) - cimag(g[c]);        /* main.c:188 */
    for (int r = 0; r < N; r++)                                          /* main.c:189, utils.c:55-65 */
        for (int c = 0; c < N; c++) Rhh[r * N + c] = g[r] * q[c];
    mat_mul(Rhh, N, N, FH, N, t1);                                       /* main.c:191 */
    mat_mul(t1, N, N, X4, N, Rhy);                                       /* main.c:192 */
    ldc ryy = (ldc)ow2 + (ldc)ow2;                                       /* main.c:198-199 */
    for (int i = 0; i < N; i++) invRyy[i * N + i] = 1.0L / ryy;          /* repair of main.c:201 */
    mat_mul(F, N, N, Rhy, N, t1);                                        /* main.c:203 */
    mat_mul(invRyy, N, N, rx, 1, t3);                                    /* main.c:204 */
    mat_mul(t1, N, N, t3, 1, H);                                         /* main.c:205 */
    free(FH); free(X4); free(Rhh); free(Rhy); free(invF); free(t1);
    free(g); free(q); free(t3); free(invRyy);
}

/* Shared (frame-independent) part of the REF-repaired MMSE:
 * C_ref = F * (Rhh * FH), so that H_f = C_ref * X4_f * rx_f / (2 ow2). */
void orc_mmse_ref_cmatrix(const ldc *F, const ldc *invF, const ldc *H_LS, ldc *C)
{
    ldc *FH = calloc(N * N, sizeof(ldc)), *Rhh = calloc(N * N, sizeof(ldc));
    ldc *t1 = calloc(N * N, sizeof(ldc)), *g = calloc(N, sizeof(ldc));
    mat_hermitian_quirk(F, N, FH);
    mat_mul(invF, N, N, H_LS, 1, g);
    for (int r = 0; r < N; r++)
        for (int c = 0; c < N; c++) Rhh[r * N + c] = g[r] * (ldc)(creal(g[c]) - cimag(g[c]));
    mat_mul(Rhh, N, N, FH, N, t1);
    mat_mul(F, N, N, t1, N, C);
    free(FH); free(Rhh); free(t1); free(g);
}

/* TEXTBOOK covariance (WiFi_channel_estimation_PS_MMSE.m:20-27):
 * Rhh = ifft(H)*ifft(H)', C = F*Rhh*F' with a true conjugate transpose. */
void orc_mmse_textbook_cmatrix(const ldc *F, const ldc *H_LS, ldc *C)
{
    ldc h[N], Fh[N];
    for (int n = 0; n < N; n++) {            /* ifft: h = conj(F) * H / N (F symmetric) */
        ldc s = 0;
        for (int k = 0; k < N; k++) s = s + conjl(F[n * N + k]) * H_LS[k];
        h[n] = s / (long double)N;
    }
    for (int i = 0; i < N; i++) {            /* F*h */
        ldc s = 0;
        for (int t = 0; t < N; t++) s = s + F[i * N + t] * h[t];
        Fh[i] = s;
    }
    for (int i = 0; i < N; i++)              /* F*(h h')*F' = (F h)(F h)' */
        for (int j = 0; j < N; j++) C[i * N + j] = Fh[i] * conjl(Fh[j]);
}

/*
 * Unified per-frame MMSE, the formula the GPU kernel implements:
 *   H = C * X * (a * X C X' + b I)^-1 * rx,   X = diag(tx .* mask)
 * REF mode: C = C_ref, mask = pilots, (a, b) = (0, 2 ow2).
 * TEXTBOOK mode: C = C_txt, mask = all, (a, b) = (1, ow2).
 * Long double Cholesky (lower, right-looking) + two triangular solves.
 */
void orc_mmse_unified(const ldc *C, const unsigned char *mask, long double a, long double b,
                      const ldc *tx, const ldc *rx, ldc *H)
{
    ldc x[N], z[N], w[N];
    ldc *A = malloc(sizeof(ldc) * N * N);
    for (int i = 0; i < N; i++) x[i] = mask[i] ? tx[i] : 0;
    for (int i = 0; i < N; i++)
        for (int j = 0; j <= i; j++)
            A[i * N + j] = a * (x[i] * C[i * N + j] * conjl(x[j])) + (i == j ? b : 0);
    for (int k = 0; k < N; k++) {
        long double d = sqrtl(creall(A[k * N + k]));
        A[k * N + k] = d;
        for (int i = k + 1; i < N; i++) A[i * N + k] /= d;
        for (int j = k + 1; j < N; j++)
            for (int i = j; i < N; i++) A[i * N + j] -= A[i * N + k] * conjl(A[j * N + k]);
    }
    for (int i = 0; i < N; i++) {             /* L y = rx */
        ldc s = rx[i];
        for (int j = 0; j < i; j++) s -= A[i * N + j] * z[j];
        z[i] = s / creall(A[i * N + i]);
    }
    for (int i = N - 1; i >= 0; i--) {        /* L' z = y */
        ldc s = z[i];
        for (int j = i + 1; j < N; j++) s -= conjl(A[j * N + i]) * w[j];
        w[i] = s / creall(A[i * N + i]);
    }
    for (int i = 0; i < N; i++) w[i] *= x[i];
    for (int i = 0; i < N; i++) {
        ldc s = 0;
        for (int j = 0; j < N; j++) s += C[i * N + j] * w[j];
        H[i] = s;
    }
    free(A);
}

/* Closed form of the TEXTBOOK MMSE when C = c c' (rank one):
 * Ryy = v v' + s I with v = X c, u = X' c, and
 * H = c * (u'rx - (u'v)(v'rx)/(s + v'v)) / s. */
void orc_mmse_textbook_closed(const ldc *c, const ldc *tx, const ldc *rx, long double s, ldc *H)
{
    ldc urx = 0, uv = 0, vrx = 0;
    long double vv = 0;
    for (int i = 0; i < N; i++) {
        ldc v = tx[i] * c[i], u = conjl(tx[i]) * c[i];
        urx += conjl(u) * rx[i];
        uv += conjl(u) * v;
        vrx += conjl(v) * rx[i];
        vv += creall(v) * creall(v) + cimagl(v) * cimagl(v);
    }
    ldc beta = (urx - uv * vrx / (s + vv)) / s;
    for (int i = 0; i < N; i++) H[i] = c[i] * beta;
}

/* WiFi_Equalization.m:1-9 (0-based block b = i-1):
 * H_UTIL = ((15-i)/15) H_LT + (i/15) H_PS; eq = rx ./ H_UTIL, DC left 0. */
void orc_equalize(const ldc *rx, const ldc *H_LT, const ldc *H_PS, ldc *eq)
{
    for (int b = 0; b < NBLK; b++) {
        long double i = b + 1;
        for (int k = 0; k < N; k++) {
            if (k == DC) { eq[b * N + k] = 0; continue; }
            ldc hu = ((NBLK - i) / NBLK) * H_LT[k] + (i / NBLK) * H_PS[k];
            eq[b * N + k] = rx[b * N + k] / hu;
        }
    }
}

/* ---- MATLAB-semantics estimators (WiFi_channel_estimation_PS_*.m): proper
 * per-block formulas, averaged over blocks 1..4.  tx/rx block-major [15][53]. */
static void avg4(void (*est)(const ldc *, const ldc *, ldc *), const ldc *tx, const ldc *rx, ldc *H)
{
    ldc t[4][N];
    for (int b = 0; b < 4; b++) est(tx + b * N, rx + b * N, t[b]);
    for (int k = 0; k < N; k++) H[k] = (t[0][k] + t[1][k] + t[2][k] + t[3][k]) / 4;
}

/* WiFi_channel_estimation_PS_Cubic.m:11-13: divisors 14, 28, 42 */
static void matlab_cubic_block(const ldc *tx, const ldc *rx, ldc *H)
{
    ldc hp[4];
    pilot_ls(tx, rx, hp);
    ldc f01 = (hp[1] - hp[0]) / 14, f12 = (hp[2] - hp[1]) / 14, f23 = (hp[3] - hp[2]) / 14;
    ldc f012 = (f12 - f01) / 28, f123 = (f23 - f12) / 28, f0123 = (f123 - f012) / 42;
    for (int k = 0; k < N; k++)
        H[k] = hp[0] + f01 * (k - P0) + f012 * (k - P0) * (k - P1)
             + f0123 * (k - P0) * (k - P1) * (k - P2);
}

void orc_matlab_ps_linear(const ldc *tx, const ldc *rx, ldc *H) { avg4(orc_ps_linear, tx, rx, H); }
void orc_matlab_ps_sinc(const ldc *tx, const ldc *rx, ldc *H) { avg4(orc_ps_sinc, tx, rx, H); }
void orc_matlab_ps_cubic(const ldc *tx, const ldc *rx, ldc *H) { avg4(matlab_cubic_block, tx, rx, H); }

/* MATLAB LT_LS (WiFi_channel_estimation_LT_LS.m): proper conjugate. */
void orc_matlab_lt_ls(const ldc *tx_pre, const ldc *rx_pre, ldc *H)
{
    for (int k = 0; k < N; k++)
        H[k] = k == DC ? 0 : (conjl(tx_pre[k]) * rx_pre[k]) / (conjl(tx_pre[k]) * tx_pre[k]);
}

/* ------------------------------------------------------------------------
 * Time-domain front end (MATLAB only; no C original).  A direct 64-point DFT
 * in long double (twiddles from cexpl), not an FFT, so the checker shares no
 * algorithm with the GPU kernel.  Pinned by matlab.mat (rx_packet -> rx_symb,
 * rx_lptot -> rx_preamble_fft).
 * ------------------------------------------------------------------------ */
#define NFFT 64         /* K            WiFi_RX.m:10 */
#define NCP 16          /* sampXblock - K, WiFi_RX.m:12 */

/* X = circshift(fft(x, 64), 26)(1:53): out[i] = DFT(x)[(i - 26) mod 64] */
static void dft64_useful(const ldc *x, ldc *out)
{
    for (int i = 0; i < N; i++) {
        const int k = (i - 26 + NFFT) % NFFT;
        ldc acc = 0;
        for (int n = 0; n < NFFT; n++)
            acc += x[n] * cexpl(-2.0L * I * acosl(-1.0L) * (long double)((n * k) % NFFT) / NFFT);
        out[i] = acc;
    }
}

/* WiFi_blocks_extraction.m:4-9: block b = samples [80 b, 80 b + 80), CP dropped */
void orc_front_blocks(const ldc *samples, int n_blocks, ldc *sym)
{
    for (int b = 0; b < n_blocks; b++) dft64_useful(samples + (NFFT + NCP) * b + NCP, sym + (long)b * N);
}

/* WiFi_RX.m:24-30: p1 = last 64 samples, p2 = the 64 before; fft of their
 * mean; ow2 = sum |p2 - p1|^2 / (2 K) */
void orc_front_preamble(const ldc *lptot, long len, ldc *pre_fft, long double *ow2)
{
    const ldc *p1 = lptot + len - NFFT, *p2 = lptot + len - 2 * NFFT;
    ldc avg[NFFT];
    long double s = 0;
    for (int n = 0; n < NFFT; n++) {
        avg[n] = (p1[n] + p2[n]) / 2;
        const ldc d = p2[n] - p1[n];
        s += creall(d * conjl(d));
    }
    dft64_useful(avg, pre_fft);
    *ow2 = s / (2 * NFFT);
}

/* ------------------------------------------------------------------------
 * fp64 batched CPU paths, OpenMP over frames.  These are the "port" CPU
 * baselines bench.py times on the GPU host (same algorithm as the GPU
 * kernels, race-free; the reference's own OpenMP path crashes).
 * Frames: tx/rx [n][frame_stride] complex, block 0 at offset 0.
 * ------------------------------------------------------------------------ */
typedef double complex dc;

double orc_bench_mmse_f64(int nthreads, const dc *C, const unsigned char *mask, double a, double b,
                          const dc *tx, const dc *rx, long n_frames, long frame_stride, dc *H)
{
    double t0 = omp_get_wtime();
#pragma omp parallel for num_threads(nthreads) schedule(static)
    for (long f = 0; f < n_frames; f++) {
        const dc *t = tx + f * frame_stride, *r = rx + f * frame_stride;
        dc A[N * N], x[N], y[N], z[N];
        for (int i = 0; i < N; i++) x[i] = mask[i] ? t[i] : 0;
        for (int i = 0; i < N; i++)
            for (int j = 0; j <= i; j++)
                A[i * N + j] = a * (x[i] * C[i * N + j] * conj(x[j])) + (i == j ? b : 0);
        for (int k = 0; k < N; k++) {
            double d = sqrt(creal(A[k * N + k])), rd = 1.0 / d;
            A[k * N + k] = d;
            for (int i = k + 1; i < N; i++) A[i * N + k] *= rd;
            for (int j = k + 1; j < N; j++) {
                dc l = conj(A[j * N + k]);
                for (int i = j; i < N; i++) A[i * N + j] -= A[i * N + k] * l;
            }
        }
        for (int i = 0; i < N; i++) {
            dc s = r[i];
            for (int j = 0; j < i; j++) s -= A[i * N + j] * y[j];
            y[i] = s / creal(A[i * N + i]);
        }
        for (int i = N - 1; i >= 0; i--) {
            dc s = y[i];
            for (int j = i + 1; j < N; j++) s -= conj(A[j * N + i]) * z[j];
            z[i] = s / creal(A[i * N + i]);
        }
        for (int i = 0; i < N; i++) z[i] *= x[i];
        for (int i = 0; i < N; i++) {
            dc s = 0;
            for (int j = 0; j < N; j++) s += C[i * N + j] * z[j];
            H[f * N + i] = s;
        }
    }
    return omp_get_wtime() - t0;
}

/* LT_LS + PS_Linear over a batch (config 2), fp64.  rx_pre [n][53] per frame,
 * tx_pre shared; pilots from block 0 of tx/rx. */
double orc_bench_ls_f64(int nthreads, const dc *tx_pre, const dc *rx_pre, const dc *tx, const dc *rx,
                        long n_frames, long frame_stride, dc *H_LT, dc *H_LIN)
{
    double t0 = omp_get_wtime();
#pragma omp parallel for num_threads(nthreads) schedule(static)
    for (long f = 0; f < n_frames; f++) {
        const dc *rp = rx_pre + f * N, *t = tx + f * frame_stride, *r = rx + f * frame_stride;
        dc *hl = H_LT + f * N, *hn = H_LIN + f * N, hp[4];
        const int P[4] = {P0, P1, P2, P3};
        for (int k = 0; k < N; k++) {
            double c = creal(tx_pre[k]) - cimag(tx_pre[k]);
            hl[k] = k == DC ? 0 : (c * rp[k]) / (c * tx_pre[k]);
        }
        for (int p = 0; p < 4; p++) hp[p] = r[P[p]] / t[P[p]];
        for (int k = 0; k < N; k++) {
            int s = k < P1 ? 0 : (k < P2 ? 1 : 2);
            double al = (k - P[s]) / 14.0;
            hn[k] = hp[s] + (hp[s + 1] - hp[s]) * al;
        }
    }
    return omp_get_wtime() - t0;
}
