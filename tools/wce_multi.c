/*
 * wce_multi.c -- a C host driving every GPU of the node from ONE process,
 * through the C ABI only (include/wce.h).  The analogue of the reference's
 * MPI driver (main_mpi.c): there, rank 0 computes F / Ryy and MPI_Bcasts them
 * (main_mpi.c:687-688, 727-728) and every rank loops over its own frames
 * (main_mpi.c:99, 140).  Here the shared state is built once on device 0 and
 * sent with ONE RCCL broadcast over xGMI (wce_ctx_broadcast_state_all), the
 * batch is sharded into contiguous frame ranges (wce_shard), and there is no
 * other exchange on the data path.
 *
 *   wce_multi [total_frames] [mode: ref|textbook] [reps] [max_devices]
 *
 * Every device generates its own frames from the global frame index (the
 * counter RNG of wce_synth_frames), so the sharded batch is the same batch a
 * single GPU would see.  Checks: every output finite (wce_nonfinite_scan,
 * combined with wce_comm_max_f64_all), and each shard's first frame
 * recomputed on device 0 alone is bit-identical.  Exit code != 0 on any
 * failure.
 */
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "wce.h"

#define CHECK(x)                                                                          \
    do {                                                                                  \
        int rc_ = (x);                                                                    \
        if (rc_) {                                                                        \
            fprintf(stderr, "%s failed: %d (%s)\n", #x, rc_, wce_last_error());           \
            exit(2);                                                                      \
        }                                                                                 \
    } while (0)

#define MAXDEV 16

static double now_s(void)
{
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return t.tv_sec + 1e-9 * t.tv_nsec;
}

struct shard {
    int dev;
    int64_t first, count;
    wce_ctx *ctx;
    wce_comm *comm;
    void *stream;
    wce_complex *tx, *rx, *H;
    uint32_t *bits;
    unsigned long long *n_bad;
};

int main(int argc, char **argv)
{
    const int64_t total = argc > 1 ? atoll(argv[1]) : 65536;
    const int mode = (argc > 2 && strcmp(argv[2], "ref") == 0) ? WCE_MMSE_REF : WCE_MMSE_TEXTBOOK;
    const int reps = argc > 3 ? atoi(argv[3]) : 20;
    const int maxdev = argc > 4 ? atoi(argv[4]) : MAXDEV;
    const double ow2 = 9.6172e-08, A = 8.8753;
    const size_t fr = (size_t)WCE_NBLK * WCE_NSC;
    int ndev = 0;
    CHECK(wce_device_count(&ndev));
    if (ndev == 0) {
        fprintf(stderr, "no device\n");
        return 1;
    }
    if (ndev > maxdev) ndev = maxdev;
    if (ndev > MAXDEV) ndev = MAXDEV;

    /* synthetic shared preamble (as tools/wce_cli.c) */
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

    struct shard sh[MAXDEV];
    int devs[MAXDEV];
    wce_comm *comms[MAXDEV];
    wce_ctx *ctxs[MAXDEV];
    void *streams[MAXDEV];
    for (int d = 0; d < ndev; d++) devs[d] = d;
    CHECK(wce_comm_init_all(comms, ndev, devs));
    for (int d = 0; d < ndev; d++) {
        struct shard *s = &sh[d];
        memset(s, 0, sizeof(*s));
        s->dev = d;
        s->comm = comms[d];
        CHECK(wce_shard(total, ndev, d, &s->first, &s->count));
        if (d == 0)
            CHECK(wce_ctx_create(&s->ctx, d, tx_pre, rx_pre, ow2, mode));   /* 80-bit host work, once */
        else
            CHECK(wce_ctx_create_empty(&s->ctx, d));
        CHECK(wce_set_device(d));
        CHECK(wce_stream_create(&s->stream));
        ctxs[d] = s->ctx;
        streams[d] = s->stream;
    }
    const double tb = now_s();
    CHECK(wce_ctx_broadcast_state_all(ctxs, comms, ndev, 0, streams));    /* the one collective */
    const double bcast_ms = (now_s() - tb) * 1e3;

    for (int d = 0; d < ndev; d++) {
        struct shard *s = &sh[d];
        const int64_t n = s->count > 0 ? s->count : 1;
        CHECK(wce_set_device(d));
        CHECK(wce_malloc((void **)&s->tx, n * fr * sizeof(wce_complex)));
        CHECK(wce_malloc((void **)&s->rx, n * fr * sizeof(wce_complex)));
        CHECK(wce_malloc((void **)&s->H, n * WCE_NSC * sizeof(wce_complex)));
        CHECK(wce_malloc((void **)&s->bits, ((n + 31) / 32) * sizeof(uint32_t)));
        CHECK(wce_malloc((void **)&s->n_bad, sizeof(unsigned long long)));
        CHECK(wce_synth_frames(s->ctx, s->tx, s->rx, NULL, fr, WCE_NSC, WCE_NSC, s->first, s->count, 0x80211ull,
                               NULL, A, ow2, s->stream));
    }
    wce_frames in[MAXDEV];
    wce_outputs out[MAXDEV];
    for (int d = 0; d < ndev; d++) {
        wce_frames f = {sh[d].tx, sh[d].rx, NULL, NULL, (int64_t)fr, WCE_NSC, WCE_NSC, sh[d].count, 0, WCE_SEM_C};
        wce_outputs o = {NULL, NULL, NULL, NULL, sh[d].H, NULL, WCE_NSC, 0, 0, 0, 0};
        in[d] = f;
        out[d] = o;
    }
    /* ~0.3 s of untimed steps (the GPUs ramp their clocks), then reps steps
     * over all devices; wall clock around both syncs */
    for (const double tw = now_s(); now_s() - tw < 0.3;) {
        for (int r = 0; r < 10; r++)
            for (int d = 0; d < ndev; d++)
                CHECK(wce_estimate(sh[d].ctx, &in[d], &out[d], WCE_EST_PS_MMSE, sh[d].stream));
        for (int d = 0; d < ndev; d++) CHECK(wce_stream_synchronize(sh[d].stream));
    }
    const double t0 = now_s();
    for (int r = 0; r < reps; r++)
        for (int d = 0; d < ndev; d++) CHECK(wce_estimate(sh[d].ctx, &in[d], &out[d], WCE_EST_PS_MMSE, sh[d].stream));
    for (int d = 0; d < ndev; d++) CHECK(wce_stream_synchronize(sh[d].stream));
    const double dt = (now_s() - t0) / reps;

    /* checks: non-finite frames (max over devices through RCCL) ... */
    double bad[MAXDEV];
    for (int d = 0; d < ndev; d++) {
        unsigned long long nb = 0;
        bad[d] = 0;
        if (sh[d].count == 0) continue;
        CHECK(wce_nonfinite_scan(sh[d].ctx, sh[d].H, WCE_NSC, sh[d].count, 0, sh[d].bits, sh[d].n_bad,
                                 sh[d].stream));
        CHECK(wce_stream_synchronize(sh[d].stream));
        CHECK(wce_set_device(d));
        CHECK(wce_memcpy_dtoh(&nb, sh[d].n_bad, sizeof(nb)));
        bad[d] = (double)nb;
    }
    CHECK(wce_comm_max_f64_all(comms, ndev, bad, streams));
    /* ... and each shard's first frame, recomputed on device 0 alone */
    int mismatches = 0;
    {
        wce_complex *tx1, *rx1, *H1, got[WCE_NSC], want[WCE_NSC];
        CHECK(wce_set_device(0));
        CHECK(wce_malloc((void **)&tx1, fr * sizeof(wce_complex)));
        CHECK(wce_malloc((void **)&rx1, fr * sizeof(wce_complex)));
        CHECK(wce_malloc((void **)&H1, WCE_NSC * sizeof(wce_complex)));
        for (int d = 0; d < ndev; d++) {
            if (sh[d].count == 0) continue;
            CHECK(wce_synth_frames(sh[0].ctx, tx1, rx1, NULL, fr, WCE_NSC, WCE_NSC, sh[d].first, 1, 0x80211ull,
                                   NULL, A, ow2, sh[0].stream));
            wce_frames f1 = {tx1, rx1, NULL, NULL, (int64_t)fr, WCE_NSC, WCE_NSC, 1, 0, WCE_SEM_C};
            wce_outputs o1 = {NULL, NULL, NULL, NULL, H1, NULL, WCE_NSC, 0, 0, 0, 0};
            CHECK(wce_estimate(sh[0].ctx, &f1, &o1, WCE_EST_PS_MMSE, sh[0].stream));
            CHECK(wce_stream_synchronize(sh[0].stream));
            CHECK(wce_memcpy_dtoh(want, H1, sizeof(want)));
            CHECK(wce_set_device(d));
            CHECK(wce_memcpy_dtoh(got, sh[d].H, sizeof(got)));
            CHECK(wce_set_device(0));
            if (memcmp(got, want, sizeof(got)) != 0) {
                fprintf(stderr, "device %d: frame %lld differs from device 0's\n", d, (long long)sh[d].first);
                mismatches++;
            }
        }
        wce_free(tx1);
        wce_free(rx1);
        wce_free(H1);
    }
    printf("wce_multi: %lld frames over %d device(s), MMSE mode %s, %s\n", (long long)total, ndev,
           mode ? "textbook" : "ref", wce_version());
    printf("  state broadcast (1 RCCL group) %.3f ms, %zu bytes\n", bcast_ms, wce_state_size());
    printf("  step %.3f ms  %.4e frames/s aggregate  (%.4e per device)\n", dt * 1e3, total / dt,
           total / dt / ndev);
    printf("  non-finite frames (max over devices): %.0f; shard-boundary frames mismatching device 0: %d\n", bad[0],
           mismatches);

    for (int d = 0; d < ndev; d++) {
        CHECK(wce_set_device(d));
        wce_free(sh[d].tx);
        wce_free(sh[d].rx);
        wce_free(sh[d].H);
        wce_free(sh[d].bits);
        wce_free(sh[d].n_bad);
        wce_stream_destroy(sh[d].stream);
        wce_ctx_destroy(sh[d].ctx);
        wce_comm_destroy(sh[d].comm);
    }
    return (bad[0] != 0 || mismatches) ? 3 : 0;
}
