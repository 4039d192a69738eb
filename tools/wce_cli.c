/*
 * wce_cli.c -- a C host that uses only the C ABI (include/wce.h): the
 * reference's driver loop (main.c:10-64) turned into a batched run.
 *
 *   wce_cli [frames] [mode: ref|textbook] [reps]
 *
 * Builds the shared state from a synthetic 802.11 preamble, generates the
 * frames (with per-frame preambles) on the device, runs LT_LS +
 * PS_Linear/Cubic/Sinc + PS_MMSE + equalization in main.c and MATLAB
 * semantics, per-frame-covariance MMSE, fp32 LS outputs and the time-domain
 * front end, and prints frames/s per configuration.  Exit code != 0 on any
 * wce error.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "wce.h"

#define CHECK(x)                                                                          \
    do {                                                                                  \
        int rc_ = (x);                                                                    \
        if (rc_) {                                                                        \
            fprintf(stderr, "%s failed: %d (%s)\n", #x, rc_, wce_last_error());           \
            exit(2);                                                                      \
        }                                                                                 \
    } while (0)

static float time_it(void *stream, wce_ctx *ctx, const wce_frames *in, const wce_outputs *out, unsigned mask,
                     int reps)
{
    void *e0, *e1;
    float ms = 0;
    CHECK(wce_estimate(ctx, in, out, mask, stream)); /* warm-up */
    CHECK(wce_event_create(&e0));
    CHECK(wce_event_create(&e1));
    CHECK(wce_event_record(e0, stream));
    for (int i = 0; i < reps; i++) CHECK(wce_estimate(ctx, in, out, mask, stream));
    CHECK(wce_event_record(e1, stream));
    CHECK(wce_event_elapsed_ms(&ms, e0, e1));
    wce_event_destroy(e0);
    wce_event_destroy(e1);
    return ms / reps;
}

int main(int argc, char **argv)
{
    const long B = argc > 1 ? atol(argv[1]) : 65536;
    const int mode = (argc > 2 && strcmp(argv[2], "textbook") == 0) ? WCE_MMSE_TEXTBOOK : WCE_MMSE_REF;
    const int reps = argc > 3 ? atoi(argv[3]) : 10;
    const double ow2 = 9.6172e-08, A = 8.8753;
    int ndev = 0;
    CHECK(wce_device_count(&ndev));
    if (ndev == 0) {
        fprintf(stderr, "no device\n");
        return 1;
    }
    /* synthetic shared preamble: BPSK long training symbol through a 3-tap channel */
    wce_complex tx_pre[WCE_NSC], rx_pre[WCE_NSC];
    for (int k = 0; k < WCE_NSC; k++) {
        double s = ((k * 7 + 3) % 5 < 2) ? -A : A;
        double th = -2 * M_PI * (k - 26) / 64.0;
        double hr = 0.009 + 0.003 * cos(th) + 0.001 * cos(2 * th), hi = 0.003 * sin(th) + 0.001 * sin(2 * th);
        tx_pre[k].re = k == WCE_DC ? 0 : s;
        tx_pre[k].im = 0;
        rx_pre[k].re = tx_pre[k].re * hr;
        rx_pre[k].im = tx_pre[k].re * hi;
    }
    wce_ctx *ctx;
    CHECK(wce_ctx_create(&ctx, 0, tx_pre, rx_pre, ow2, mode));
    void *stream;
    CHECK(wce_stream_create(&stream));
    const size_t fr = (size_t)WCE_NBLK * WCE_NSC;
    wce_complex *tx, *rx, *pre, *h[5], *eq;
    CHECK(wce_malloc((void **)&tx, B * fr * sizeof(wce_complex)));
    CHECK(wce_malloc((void **)&rx, B * fr * sizeof(wce_complex)));
    CHECK(wce_malloc((void **)&pre, B * WCE_NSC * sizeof(wce_complex)));
    CHECK(wce_malloc((void **)&eq, B * fr * sizeof(wce_complex)));
    for (int i = 0; i < 5; i++) CHECK(wce_malloc((void **)&h[i], B * WCE_NSC * sizeof(wce_complex)));
    CHECK(wce_synth_frames(ctx, tx, rx, pre, fr, WCE_NSC, WCE_NSC, 0, B, 0x80211ull, NULL, A, ow2, stream));
    CHECK(wce_ctx_reserve(ctx, B));
    wce_frames in = {tx, rx, NULL, NULL, (int64_t)fr, WCE_NSC, WCE_NSC, B, 0, WCE_SEM_C};
    wce_frames in_pre = {tx, rx, pre, NULL, (int64_t)fr, WCE_NSC, WCE_NSC, B, 0, WCE_SEM_C};
    wce_frames in_ml = {tx, rx, pre, NULL, (int64_t)fr, WCE_NSC, WCE_NSC, B, 0, WCE_SEM_MATLAB};
    wce_outputs out = {h[0], h[1], h[2], h[3], h[4], eq, WCE_NSC, (int64_t)fr, WCE_NSC, 0, 0};
    wce_outputs out32 = out;
    out32.flags = WCE_OUT_LS_F32;   /* same buffers, half the bytes used */
    const unsigned all = WCE_EST_LS_ALL | WCE_EST_PS_MMSE | WCE_EQUALIZE;
    struct { const char *name; const wce_frames *in; const wce_outputs *out; unsigned mask; } cfg[] = {
        {"LT_LS+PS_Linear (per-frame preamble)", &in_pre, &out, WCE_EST_LT_LS | WCE_EST_PS_LINEAR},
        {"LS family (4 estimators)", &in, &out, WCE_EST_LS_ALL},
        {"PS_MMSE", &in, &out, WCE_EST_PS_MMSE},
        {"PS_MMSE per-frame covariance", &in_pre, &out, WCE_EST_PS_MMSE | WCE_MMSE_FRAME_COV},
        {"all 5 + equalization (fused)", &in_pre, &out, all},
        {"all 5 + eq, fp32 LS outputs", &in_pre, &out32, all},
        {"all 5 + eq, MATLAB semantics", &in_ml, &out, all},
    };
    printf("wce_cli: %ld frames, MMSE mode %s, %s\n", B, mode ? "textbook" : "ref", wce_version());
    for (unsigned c = 0; c < sizeof(cfg) / sizeof(cfg[0]); c++) {
        float ms = time_it(stream, ctx, cfg[c].in, cfg[c].out, cfg[c].mask, reps);
        printf("  %-38s %9.3f ms  %.3e frames/s\n", cfg[c].name, ms, B / (ms * 1e-3));
    }
    /* time-domain front end (WiFi_blocks_extraction.m): 15 x 80 samples per frame */
    {
        const size_t ns = (size_t)WCE_NBLK * WCE_SAMPLES_PER_BLOCK;
        wce_complex *samples, *lptot;
        double *sig2;
        CHECK(wce_malloc((void **)&samples, B * ns * sizeof(wce_complex)));
        CHECK(wce_malloc((void **)&lptot, B * 160 * sizeof(wce_complex)));
        CHECK(wce_malloc((void **)&sig2, B * sizeof(double)));
        CHECK(wce_memset(samples, 0, B * ns * sizeof(wce_complex)));
        CHECK(wce_memset(lptot, 0, B * 160 * sizeof(wce_complex)));
        void *e0, *e1;
        float ms = 0;
        CHECK(wce_event_create(&e0));
        CHECK(wce_event_create(&e1));
        CHECK(wce_front_end_blocks(ctx, samples, (int64_t)ns, B, WCE_NBLK, rx, (int64_t)fr, WCE_NSC, stream));
        CHECK(wce_event_record(e0, stream));
        for (int i = 0; i < reps; i++) {
            CHECK(wce_front_end_preamble(ctx, lptot, 160, 160, B, pre, WCE_NSC, sig2, stream));
            CHECK(wce_front_end_blocks(ctx, samples, (int64_t)ns, B, WCE_NBLK, rx, (int64_t)fr, WCE_NSC, stream));
        }
        CHECK(wce_event_record(e1, stream));
        CHECK(wce_event_elapsed_ms(&ms, e0, e1));
        ms /= reps;
        printf("  %-38s %9.3f ms  %.3e frames/s\n", "front end (LTF + 15 blocks)", ms, B / (ms * 1e-3));
        wce_event_destroy(e0);
        wce_event_destroy(e1);
        wce_free(samples);
        wce_free(lptot);
        wce_free(sig2);
    }
    /* the reference's own data format (long double complex, main.c:4-8): raw
       x87 bytes to the device, converted there; every value must equal this
       compiler's C casts bit for bit, both ways */
    {
        const long nv = (B < 4096 ? B : 4096) * (long)fr;
        long double _Complex *hld = malloc(nv * sizeof(*hld)), *back = malloc(nv * sizeof(*back));
        wce_complex *hc = malloc(nv * sizeof(*hc));
        if (!hld || !back || !hc) {
            fprintf(stderr, "host alloc\n");
            return 4;
        }
        for (long i = 0; i < nv; i++) {   /* bits below fp64, so (double) must round */
            long double re = A * sinl(0.37L * i) * (1 + 0x1p-60L * (i % 7));
            long double im = A * cosl(0.11L * i) * (1 - 0x1p-61L * (i % 5));
            __real__ hld[i] = re;
            __imag__ hld[i] = im;
        }
        void *dld;
        wce_complex *dc;
        CHECK(wce_malloc(&dld, nv * sizeof(*hld)));
        CHECK(wce_malloc((void **)&dc, nv * sizeof(*hc)));
        CHECK(wce_memcpy_htod(dld, hld, nv * sizeof(*hld)));
        CHECK(wce_ldc_to_complex(dld, dc, nv, stream));
        CHECK(wce_complex_to_ldc(dc, dld, nv, stream));
        CHECK(wce_stream_synchronize(stream));
        CHECK(wce_memcpy_dtoh(hc, dc, nv * sizeof(*hc)));
        CHECK(wce_memcpy_dtoh(back, dld, nv * sizeof(*back)));
        long bad = 0;
        for (long i = 0; i < nv; i++) {
            const double re = (double)__real__ hld[i], im = (double)__imag__ hld[i];
            const long double bre = re, bim = im;
            bad += memcmp(&re, &hc[i].re, 8) != 0 || memcmp(&im, &hc[i].im, 8) != 0;
            bad += memcmp(&bre, &__real__ back[i], 10) != 0 || memcmp(&bim, &__imag__ back[i], 10) != 0;
        }
        if (bad) {
            fprintf(stderr, "long double conversion: %ld mismatches\n", bad);
            return 4;
        }
        printf("  %-38s %ld values, bit-identical to the C casts\n", "long double complex <-> device", nv);
        wce_free(dld);
        wce_free(dc);
        free(hld);
        free(back);
        free(hc);
    }
    /* WCE_MMSE_COV with a model covariance: a 6-tap exponential power-delay
     * profile (rank 6) takes the low-rank Gram path; an indefinite Rhh is refused */
    {
        static wce_complex R[WCE_NSC * WCE_NSC];
        double norm = 0;
        for (int t = 0; t < 6; t++) norm += exp(-0.5 * t);
        for (int t = 0; t < 6; t++) R[t * WCE_NSC + t].re = 1.1e-4 * exp(-0.5 * t) / norm;
        wce_ctx *cov;
        CHECK(wce_ctx_create_cov(&cov, 0, tx_pre, rx_pre, R, ow2));
        int rank = -1, lowrank = -1;
        double lmax = 0, lmin = 0;
        CHECK(wce_ctx_cov_info(cov, &rank, &lowrank, &lmax, &lmin));
        if (rank != 6 || lowrank != 1) {
            fprintf(stderr, "cov info: rank %d low-rank %d\n", rank, lowrank);
            return 4;
        }
        float ms = time_it(stream, cov, &in, &out, WCE_EST_PS_MMSE, reps);
        printf("  %-38s %9.3f ms  %.3e frames/s (rank %d, low-rank path)\n", "PS_MMSE, 6-tap PDP covariance", ms,
               B / (ms * 1e-3), rank);
        CHECK(wce_ctx_destroy(cov));
        R[3 * WCE_NSC + 3].re = -1e-6;   /* indefinite: must be refused */
        if (wce_ctx_create_cov(&cov, 0, tx_pre, rx_pre, R, ow2) != WCE_EINVAL) {
            fprintf(stderr, "indefinite Rhh accepted\n");
            return 5;
        }
    }
    /* spot check: LT_LS of frame 0 at DC must be 0 (main.c:74) */
    wce_complex h0[WCE_NSC];
    CHECK(wce_stream_synchronize(stream));
    CHECK(wce_memcpy_dtoh(h0, h[0], sizeof(h0)));
    if (h0[WCE_DC].re != 0 || h0[WCE_DC].im != 0) {
        fprintf(stderr, "DC not zero\n");
        return 3;
    }
    for (int i = 0; i < 5; i++) wce_free(h[i]);
    wce_free(pre);
    wce_free(tx);
    wce_free(rx);
    wce_free(eq);
    wce_stream_destroy(stream);
    wce_ctx_destroy(ctx);
    return 0;
}
