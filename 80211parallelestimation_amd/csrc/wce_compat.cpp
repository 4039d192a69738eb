// wce_compat.cpp -- the reference's five entry points (main.c:4-8) on top of
// the batched C ABI: one frame, host long double _Complex arrays in/out,
// fp64 on the GPU.  Compiled by g++ (x87 long double, like the reference).
#include <cstring>
#include <mutex>

#include "../../include/wce_compat.h"
#include "wce_internal.h"

namespace {

typedef __complex__ long double cld;

constexpr int SLOT = 64;
enum { S_TX, S_RX, S_RXPRE, S_TXPRE, S_LT, S_LIN, S_CUB, S_SNC, S_MMSE, S_COUNT };

struct CompatEngine {
    wce_ctx *ctx = nullptr;
    wce_complex *d = nullptr;        // S_COUNT slots of 64 complex
    wce::State host;                 // state currently on the device
    bool host_valid = false;
    // main.c:148's shared inputs of the last PS_MMSE call: a caller looping
    // frames with one preamble (main.c:53 computes H_EST_LS once) reuses the
    // state already on the device instead of rebuilding and re-uploading it
    bool mmse_valid = false;
    wce::ldc last_F[wce::NSC * wce::NSC], last_hls[wce::NSC];
    double last_ow2 = 0.0;
    unsigned long long state_builds = 0;
};

std::mutex g_mu;
CompatEngine *g_eng = nullptr;
int g_last = WCE_OK;

// long double has padding bytes: compare values, not memory (a NaN never
// compares equal, so such inputs always rebuild)
bool same_ldc(const wce::ldc *a, const wce::ldc *b, int n)
{
    for (int i = 0; i < n; i++)
        if (!(a[i].re == b[i].re && a[i].im == b[i].im)) return false;
    return true;
}

int upload(CompatEngine &e)
{
    void *dst = nullptr;
    size_t bytes = 0;
    int rc = wce_ctx_state(e.ctx, &dst, &bytes);
    if (rc) return rc;
    rc = wce_memcpy_htod(dst, &e.host, sizeof(wce::State));
    if (rc) return rc;
    return wce_ctx_mark_ready(e.ctx);
}

int engine(CompatEngine **out)
{
    if (g_eng) { *out = g_eng; return WCE_OK; }
    CompatEngine *e = new CompatEngine;
    int rc = wce_ctx_create_empty(&e->ctx, 0);
    if (!rc) rc = wce_malloc(reinterpret_cast<void **>(&e->d), sizeof(wce_complex) * SLOT * S_COUNT);
    if (!rc) rc = wce_memset(e->d, 0, sizeof(wce_complex) * SLOT * S_COUNT);
    if (!rc) {
        // neutral state for the LS entry points (they supply their own preamble)
        wce::ldc zero[wce::NSC];
        std::memset(zero, 0, sizeof(zero));
        rc = wce::host_build_state(&e->host, wce::host_reference_F(), wce::host_reference_invF(), zero, zero, 1.0,
                                   WCE_MMSE_REF);
    }
    if (!rc) rc = upload(*e);
    if (rc) {
        if (e->d) wce_free(e->d);
        if (e->ctx) wce_ctx_destroy(e->ctx);
        delete e;
        return rc;
    }
    e->host_valid = true;
    g_eng = e;
    *out = e;
    return WCE_OK;
}

void to_dev(CompatEngine &e, int slot, const long double _Complex *v, int &rc)
{
    if (rc) return;
    wce_complex h[SLOT];
    std::memset(h, 0, sizeof(h));
    for (int k = 0; k < wce::NSC; k++) {
        h[k].re = (double)__real__ v[k];
        h[k].im = (double)__imag__ v[k];
    }
    rc = wce_memcpy_htod(e.d + slot * SLOT, h, sizeof(h));
}

void from_dev(CompatEngine &e, int slot, long double _Complex *v, int &rc)
{
    if (rc) return;
    wce_complex h[SLOT];
    rc = wce_memcpy_dtoh(h, e.d + slot * SLOT, sizeof(h));
    if (rc) return;
    for (int k = 0; k < wce::NSC; k++) {
        cld z;
        __real__ z = h[k].re;
        __imag__ z = h[k].im;
        v[k] = z;
    }
}

// One frame through wce_estimate: tx/rx are block 0 of the frame.
int run_one(uint32_t mask, const long double _Complex *tx, const long double _Complex *rx, int out_slot,
            long double _Complex *H, bool preamble)
{
    CompatEngine *e = nullptr;
    int rc = engine(&e);
    if (rc) return rc;
    to_dev(*e, preamble ? S_TXPRE : S_TX, tx, rc);
    to_dev(*e, preamble ? S_RXPRE : S_RX, rx, rc);
    if (rc) return rc;
    wce_frames in;
    std::memset(&in, 0, sizeof(in));
    in.tx = e->d + S_TX * SLOT;
    in.rx = e->d + S_RX * SLOT;
    in.rx_pre = preamble ? e->d + S_RXPRE * SLOT : nullptr;
    in.tx_pre = preamble ? e->d + S_TXPRE * SLOT : nullptr;
    in.frame_stride = SLOT;
    in.block_stride = SLOT;
    in.pre_stride = SLOT;
    in.n_frames = 1;
    wce_outputs out;
    std::memset(&out, 0, sizeof(out));
    out.lt_ls = e->d + S_LT * SLOT;
    out.ps_linear = e->d + S_LIN * SLOT;
    out.ps_cubic = e->d + S_CUB * SLOT;
    out.ps_sinc = e->d + S_SNC * SLOT;
    out.ps_mmse = e->d + S_MMSE * SLOT;
    out.out_stride = SLOT;
    rc = wce_estimate(e->ctx, &in, &out, mask, nullptr);
    if (!rc) rc = wce_stream_synchronize(nullptr);
    from_dev(*e, out_slot, H, rc);
    return rc;
}

}  // namespace

extern "C" {

int wce_compat_last_status(void) { return g_last; }

unsigned long long wce_debug_compat_state_builds(void)
{
    std::lock_guard<std::mutex> lk(g_mu);
    return g_eng ? g_eng->state_builds : 0ULL;
}

void WiFi_channel_estimation_LT_LS(long double _Complex tx_pre[], long double _Complex rx_pre[],
                                   long double _Complex H_EST[])
{
    std::lock_guard<std::mutex> lk(g_mu);
    g_last = run_one(WCE_EST_LT_LS, tx_pre, rx_pre, S_LT, H_EST, true);
}

void WiFi_channel_estimation_PS_Linear(long double _Complex tx[], long double _Complex rx[],
                                       long double _Complex H_EST[])
{
    std::lock_guard<std::mutex> lk(g_mu);
    g_last = run_one(WCE_EST_PS_LINEAR, tx, rx, S_LIN, H_EST, false);
}

void WiFi_channel_estimation_PS_Cubic(long double _Complex tx[], long double _Complex rx[],
                                      long double _Complex H_EST[])
{
    std::lock_guard<std::mutex> lk(g_mu);
    g_last = run_one(WCE_EST_PS_CUBIC, tx, rx, S_CUB, H_EST, false);
}

void WiFi_channel_estimation_PS_Sinc(long double _Complex tx[], long double _Complex rx[],
                                     long double _Complex H_EST[])
{
    std::lock_guard<std::mutex> lk(g_mu);
    g_last = run_one(WCE_EST_PS_SINC, tx, rx, S_SNC, H_EST, false);
}

// main.c:148: the shared state (invF of the caller's F, C_ref from H_EST_LS)
// is built on the host in 80-bit arithmetic and uploaded when (F, H_EST_LS,
// ow2) differ from the previous call's; the per-frame solve and product run
// on the GPU.  invF is precomputed for the standard F.
void WiFi_channel_estimation_PS_MMSE(long double _Complex tx[], long double _Complex rx[],
                                     long double _Complex **F, double ow2, long double _Complex H_EST_LS[],
                                     long double _Complex H_EST[])
{
    std::lock_guard<std::mutex> lk(g_mu);
    CompatEngine *e = nullptr;
    int rc = engine(&e);
    if (rc) { g_last = rc; return; }
    const int n = wce::NSC;
    static wce::ldc Fl[wce::NSC * wce::NSC], invF[wce::NSC * wce::NSC];
    for (int r = 0; r < n; r++)
        for (int c = 0; c < n; c++) {
            Fl[r * n + c].re = __real__ F[r][c];
            Fl[r * n + c].im = __imag__ F[r][c];
        }
    wce::ldc hls[wce::NSC], txp[wce::NSC];
    for (int k = 0; k < n; k++) {
        hls[k].re = __real__ H_EST_LS[k];
        hls[k].im = __imag__ H_EST_LS[k];
        txp[k].re = e->host.tx_pre[2 * k];
        txp[k].im = e->host.tx_pre[2 * k + 1];
    }
    if (!(e->mmse_valid && ow2 == e->last_ow2 && same_ldc(hls, e->last_hls, n) && same_ldc(Fl, e->last_F, n * n))) {
        e->mmse_valid = false;
        const wce::ldc *Fref = wce::host_reference_F();
        const wce::ldc *inv = wce::host_reference_invF();
        if (!same_ldc(Fl, Fref, n * n)) {   // caller's own F: recompute the cofactor inverse
            wce::host_inverse_cofactor(Fl, n, invF, 8);
            inv = invF;
        }
        rc = wce::host_build_state(&e->host, Fl, inv, hls, txp, ow2, WCE_MMSE_REF);
        if (!rc) rc = upload(*e);
        if (!rc) {
            e->state_builds++;
            std::memcpy(e->last_F, Fl, sizeof(Fl));
            std::memcpy(e->last_hls, hls, sizeof(hls));
            e->last_ow2 = ow2;
            e->mmse_valid = true;
        }
    }
    if (!rc) rc = run_one(WCE_EST_PS_MMSE, tx, rx, S_MMSE, H_EST, false);
    g_last = rc;
}

}  // extern "C"
