// ref_harness.cpp -- TEST INFRASTRUCTURE ONLY (builds oracle/_ref/libref.so).
//
// Compiles the reference's own main.c / utils.c from where they lie under
// /root/reference (never copied) and exposes their estimator functions and
// matrix helpers through extern "C" entry points, so tests/golden/make_golden.py
// can produce golden vectors from the real reference code.  Built with
// g++ -std=gnu++98 against the MPICH headers the image ships in /opt/conda
// (utils.h includes <mpi.h>); recipe in oracle/Makefile.
#define main ref_main
#include "main.c"
#undef main

#include <stdlib.h>

typedef long double complex ldc;

static ldc **rows(ldc *flat, int n, int m)
{
    ldc **r = (ldc **)malloc(sizeof(ldc *) * n);
    for (int i = 0; i < n; i++) r[i] = flat + (size_t)i * m;
    return r;
}

extern "C" {

// inputs.h globals (inputs.h:18,20,75,130,928)
double refh_ow2(void) { return OW2; }
void refh_inputs(ldc *tx_pre, ldc *rx_pre, ldc *tx_sym, ldc *rx_sym)
{
    for (int i = 0; i < SAMPUTIL; i++) { tx_pre[i] = tx_preamble_fft[i]; rx_pre[i] = rx_preamble_fft[i]; }
    for (int i = 0; i < SIZESYMBOL; i++) { tx_sym[i] = tx_symb[i]; rx_sym[i] = rx_symb[i]; }
}

// main.c:18-26 (same expression, evaluated by the reference's compiler settings)
void refh_fmatrix(ldc *F)
{
    for (int f = 0; f < SAMPUTIL; f++)
        for (int t = 0; t < SAMPUTIL; t++)
            F[t * SAMPUTIL + f] = cexp(-2 * I * PI * t * f / SAMPUTIL);
}

void refh_lt_ls(ldc *tx, ldc *rx, ldc *H) { WiFi_channel_estimation_LT_LS(tx, rx, H); }
void refh_ps_linear(ldc *tx, ldc *rx, ldc *H) { WiFi_channel_estimation_PS_Linear(tx, rx, H); }
void refh_ps_cubic(ldc *tx, ldc *rx, ldc *H) { WiFi_channel_estimation_PS_Cubic(tx, rx, H); }
void refh_ps_sinc(ldc *tx, ldc *rx, ldc *H) { WiFi_channel_estimation_PS_Sinc(tx, rx, H); }

// utils.c:141 inverse (cofactor / unpivoted Schur determinant)
void refh_inverse(ldc *A, int n, ldc *Y)
{
    ldc **a = rows(A, n, n), **y = rows(Y, n, n);
    inverse(a, n, y);
    free(a); free(y);
}

// utils.c:543 determinant_impl_rec
void refh_det(ldc *A, int n, ldc *out)
{
    ldc **a = rows(A, n, n);
    *out = determinant_impl_rec(a, n);
    free(a);
}

// The reference's PS_MMSE (main.c:148-212) rebuilt from the reference's own
// helpers in the same order, with the single repair: invRyy = exact inverse
// of the diagonal Ryy (the cofactor inverse returns NaN off the diagonal).
// invF_in != NULL skips the 4 s inverse(F) (pass the reference's own invF).
void refh_mmse_repaired(ldc *tx_symbols, ldc *rx_symbols, ldc *Fflat, double ow2,
                        ldc *H_EST_LS, ldc *invF_in, ldc *H_EST_MMSE, ldc *invF_out)
{
    const int n = SAMPUTIL;
    ldc *buf = (ldc *)calloc((size_t)n * n * 12 + 4 * n, sizeof(ldc));
    ldc **F = rows(Fflat, n, n);
    ldc **FHermitian = rows(buf + 0 * n * n, n, n), **X4Hermitian = rows(buf + 1 * n * n, n, n);
    ldc **X4 = rows(buf + 2 * n * n, n, n), **Rhh = rows(buf + 3 * n * n, n, n);
    ldc **Rhy = rows(buf + 4 * n * n, n, n), **Ryy = rows(buf + 5 * n * n, n, n);
    ldc **invRyy = rows(buf + 6 * n * n, n, n), **invF = rows(buf + 7 * n * n, n, n);
    ldc **temp1 = rows(buf + 8 * n * n, n, n), **temp2 = rows(buf + 9 * n * n, n, n);
    ldc **temp3 = rows(buf + 10 * n * n, n, n), **Id = rows(buf + 11 * n * n, n, n);
    ldc **rx1 = rows(buf + 12 * n * n, n, 1), **H1 = rows(buf + 12 * n * n + n, n, 1);
    for (int r = 0; r < n; r++) {
        for (int c = 0; c < n; c++) {
            if (r == c && (r == P0 || r == P1 || r == P2 || r == P3)) X4[r][c] = tx_symbols[r];
            else X4[r][c] = 0.0;
        }
        rx1[r][0] = rx_symbols[r];
        H1[r][0] = H_EST_LS[r];
    }
    hermitian(F, n, n, FHermitian);
    hermitian(X4, n, n, X4Hermitian);
    if (invF_in) { for (int i = 0; i < n * n; i++) invF[i / n][i % n] = invF_in[i]; }
    else inverse(F, n, invF);
    if (invF_out) for (int i = 0; i < n * n; i++) invF_out[i] = invF[i / n][i % n];
    multiply(invF, n, n, H1, n, 1, temp1);
    hermitian(temp1, n, n, temp2);      // only row 0 of temp2 is consumed below
    multiplyVxVeqM(temp1, n, n, temp2, n, n, Rhh);
    multiply(Rhh, n, n, FHermitian, n, n, temp1);
    multiply(temp1, n, n, X4, n, n, Rhy);
    identity(Id, n, ow2);
    addition(Id, n, n, temp2, n, n, Ryy);
    for (int r = 0; r < n; r++)
        for (int c = 0; c < n; c++) invRyy[r][c] = (r == c) ? 1.0L / Ryy[r][c] : 0.0L;  // repair
    multiply(F, n, n, Rhy, n, n, temp1);
    multiply(invRyy, n, n, rx1, n, 1, temp3);
    multiply(temp1, n, n, temp3, n, 1, temp2);
    for (int r = 0; r < n; r++) H_EST_MMSE[r] = temp2[r][0];
    free(F); free(FHermitian); free(X4Hermitian); free(X4); free(Rhh); free(Rhy); free(Ryy);
    free(invRyy); free(invF); free(temp1); free(temp2); free(temp3); free(Id); free(rx1); free(H1);
    free(buf);
}

// WiFi_channel_estimation_PS_MMSE.m:26-33 (one block), composed from the
// reference's own matrix routines: multiply() (utils.c:16-31) for every
// product and inverse() (utils.c:141-170, the cofactor / unpivoted-Schur
// inverse) for pinv(Ryy), all in its long double complex.  The reference has
// no conjugate transpose (its hermitian() is re - im, utils.c:3-7), so the
// .m file's ' is formed here, and the MATLAB ifft is conj(F) h / 53.
//   C   : Rhh_in == NULL -> Rhh = ifft(H_LS) ifft(H_LS)' (TEXTBOOK); else the
//         caller's 53 x 53 Rhh (WCE_MMSE_COV); C = F Rhh F'.
//   Ryy = X4 C X4' + ow2 I, X4 = diag(tx);  H = F (Rhh F' X4) inv(Ryy) rx.
// One step differs from calling inverse(Ryy) on all 53: a null subcarrier
// (tx = 0, e.g. DC) leaves Ryy's row and column = ow2 e_i, and the cofactor
// of a minor with that column but not that row is 0/0 in the unpivoted
// Schur recursion (the NaN of main.c's PS_MMSE).  Ryy is block
// diagonal there, so inverse() runs on the block of the other subcarriers
// and the null's entry is 1 / ow2 -- the same inverse, exactly.
void refh_mmse_formula(ldc *tx, ldc *rx, ldc *Fflat, double ow2, ldc *H_LS, ldc *Rhh_in, ldc *H_out)
{
    const int n = SAMPUTIL;
    ldc *buf = (ldc *)calloc((size_t)n * n * 10 + 4 * n, sizeof(ldc));
    ldc **F = rows(Fflat, n, n);
    ldc **FH = rows(buf + 0 * n * n, n, n), **Fc = rows(buf + 1 * n * n, n, n);
    ldc **Rhh = rows(buf + 2 * n * n, n, n), **C = rows(buf + 3 * n * n, n, n);
    ldc **X4 = rows(buf + 4 * n * n, n, n), **X4H = rows(buf + 5 * n * n, n, n);
    ldc **T1 = rows(buf + 6 * n * n, n, n), **Ryy = rows(buf + 7 * n * n, n, n);
    ldc **Rhy = rows(buf + 8 * n * n, n, n), **invRyy = rows(buf + 9 * n * n, n, n);
    ldc **hv = rows(buf + 10 * n * n, n, 1), **hls = rows(buf + 10 * n * n + n, n, 1);
    ldc **rx1 = rows(buf + 10 * n * n + 2 * n, n, 1), **tmp = rows(buf + 10 * n * n + 3 * n, n, 1);
    for (int r = 0; r < n; r++)
        for (int c = 0; c < n; c++) {
            FH[r][c] = conjl(F[c][r]);
            Fc[r][c] = conjl(F[r][c]);
            X4[r][c] = r == c ? tx[r] : 0.0L;
            X4H[r][c] = r == c ? conjl(tx[r]) : 0.0L;
        }
    for (int r = 0; r < n; r++) { hls[r][0] = H_LS ? H_LS[r] : 0.0L; rx1[r][0] = rx[r]; }
    if (Rhh_in) {
        for (int i = 0; i < n * n; i++) Rhh[i / n][i % n] = Rhh_in[i];
    } else {
        multiply(Fc, n, n, hls, n, 1, hv);                       // ifft(H_LS, 53) * 53
        for (int r = 0; r < n; r++) hv[r][0] = hv[r][0] / (long double)n;
        for (int r = 0; r < n; r++)
            for (int c = 0; c < n; c++) Rhh[r][c] = hv[r][0] * conjl(hv[c][0]);
    }
    multiply(Rhh, n, n, FH, n, n, T1);
    multiply(F, n, n, T1, n, n, C);                              // C = F Rhh F'
    multiply(X4, n, n, C, n, n, T1);
    multiply(T1, n, n, X4H, n, n, Ryy);                          // X4 C X4'
    for (int r = 0; r < n; r++) Ryy[r][r] = Ryy[r][r] + (long double)ow2;
    int keep[SAMPUTIL], m = 0;
    for (int r = 0; r < n; r++)
        if (tx[r] != 0.0L) keep[m++] = r;
    for (int r = 0; r < n; r++)
        for (int c = 0; c < n; c++) invRyy[r][c] = 0.0L;
    for (int r = 0; r < n; r++)
        if (tx[r] == 0.0L) invRyy[r][r] = 1.0L / Ryy[r][r];
    if (m > 0) {
        ldc *sb = (ldc *)calloc((size_t)2 * m * m, sizeof(ldc));
        ldc **S = rows(sb, m, m), **Si = rows(sb + (size_t)m * m, m, m);
        for (int r = 0; r < m; r++)
            for (int c = 0; c < m; c++) S[r][c] = Ryy[keep[r]][keep[c]];
        inverse(S, m, Si);                                       // utils.c:141 on the coupled block
        for (int r = 0; r < m; r++)
            for (int c = 0; c < m; c++) invRyy[keep[r]][keep[c]] = Si[r][c];
        free(S); free(Si); free(sb);
    }
    multiply(Rhh, n, n, FH, n, n, T1);
    multiply(T1, n, n, X4, n, n, Rhy);                           // Rhy = Rhh F' X4
    multiply(invRyy, n, n, rx1, n, 1, tmp);                      // inv(Ryy) rx
    multiply(Rhy, n, n, tmp, n, 1, hv);
    multiply(F, n, n, hv, n, 1, tmp);                            // F Rhy inv(Ryy) rx
    for (int r = 0; r < n; r++) H_out[r] = tmp[r][0];
    free(F); free(FH); free(Fc); free(Rhh); free(C); free(X4); free(X4H); free(T1); free(Ryy); free(Rhy);
    free(invRyy); free(hv); free(hls); free(rx1); free(tmp);
    free(buf);
}

// ---- CPU baselines timed by bench.py (the reference's own sequential code) ----
// Frames are [n][53] long double complex.  Return wall seconds.

// LT_LS (per-frame preamble) + PS_Linear: BASELINE configs[1], main.c:66-101
double refh_bench_ls(int n, ldc *tx_pre, ldc *rx_pre, ldc *tx, ldc *rx, ldc *H_lt, ldc *H_lin)
{
    const double t0 = omp_get_wtime();
    for (int f = 0; f < n; f++) {
        const size_t o = (size_t)f * SAMPUTIL;
        WiFi_channel_estimation_LT_LS(tx_pre, rx_pre + o, H_lt + o);
        WiFi_channel_estimation_PS_Linear(tx + o, rx + o, H_lin + o);
    }
    return omp_get_wtime() - t0;
}

// PS_MMSE, main.c:148-212 with its own matrix routines, the NaN inverse(Ryy)
// repaired and the per-frame 4-s inverse(F) hoisted (invF given): REF mode
double refh_bench_mmse(int n, ldc *tx, ldc *rx, ldc *F, double ow2, ldc *H_ls, ldc *invF, ldc *H)
{
    const double t0 = omp_get_wtime();
    for (int f = 0; f < n; f++) {
        const size_t o = (size_t)f * SAMPUTIL;
        refh_mmse_repaired(tx + o, rx + o, F, ow2, H_ls, invF, H + o, NULL);
    }
    return omp_get_wtime() - t0;
}

// The same two loops with the frames split over `threads` OpenMP threads:
// the reference's per-frame functions touch only their own arguments (and
// malloc), so a frames-parallel loop over them is race-free -- unlike the
// reference's own OpenMP driver (main_openmp.c), which crashes.
double refh_bench_ls_omp(int n, int threads, ldc *tx_pre, ldc *rx_pre, ldc *tx, ldc *rx, ldc *H_lt, ldc *H_lin)
{
    const double t0 = omp_get_wtime();
#pragma omp parallel for num_threads(threads) schedule(static)
    for (int f = 0; f < n; f++) {
        const size_t o = (size_t)f * SAMPUTIL;
        WiFi_channel_estimation_LT_LS(tx_pre, rx_pre + o, H_lt + o);
        WiFi_channel_estimation_PS_Linear(tx + o, rx + o, H_lin + o);
    }
    return omp_get_wtime() - t0;
}

double refh_bench_mmse_omp(int n, int threads, ldc *tx, ldc *rx, ldc *F, double ow2, ldc *H_ls, ldc *invF, ldc *H)
{
    const double t0 = omp_get_wtime();
#pragma omp parallel for num_threads(threads) schedule(dynamic, 1)
    for (int f = 0; f < n; f++) {
        const size_t o = (size_t)f * SAMPUTIL;
        refh_mmse_repaired(tx + o, rx + o, F, ow2, H_ls, invF, H + o, NULL);
    }
    return omp_get_wtime() - t0;
}

// TEXTBOOK PS_MMSE (WiFi_channel_estimation_PS_MMSE.m:26-33, the bench's
// headline mode) through the reference's own multiply() and cofactor
// inverse() (refh_mmse_formula above), frames split over `threads` OpenMP
// threads (1 = sequential).  Each frame inverts its own 52 x 52 Ryy with the
// reference's O(n^5) cofactor routine (~4 s per frame on one core).
double refh_bench_mmse_formula(int n, int threads, ldc *tx, ldc *rx, ldc *F, double ow2, ldc *H_ls, ldc *H)
{
    const double t0 = omp_get_wtime();
#pragma omp parallel for num_threads(threads) schedule(dynamic, 1)
    for (int f = 0; f < n; f++) {
        const size_t o = (size_t)f * SAMPUTIL;
        refh_mmse_formula(tx + o, rx + o, F, ow2, H_ls, NULL, H + o);
    }
    return omp_get_wtime() - t0;
}

}  // extern "C"
