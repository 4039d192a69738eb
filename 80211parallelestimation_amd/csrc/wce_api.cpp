// wce_api.cpp -- C ABI (include/wce.h): context lifetime, argument checks,
// launches, and thin HIP runtime helpers.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "wce_internal.h"

using wce::State;

struct wce_ctx {
    int device = 0;
    State *d_state = nullptr;   // device-resident shared state (the broadcast unit)
    bool ready = false;
    bool has_host = false;
    State host;                 // host copy when built locally
    int32_t mode = -1;          // State::mode, cached when the state becomes valid
    bool fuse = true;           // config-5 fusion (wce_debug_set_fusion turns it off for A/B)
    bool bdot = true;           // rank-1 C: second bordered row, no back-solve / GEMM (A/B switch)
    int32_t cov_k0 = -1;        // State::cov_k0 (WCE_MMSE_COV: >= 0 low-rank Gram path, -1 dense)
    int32_t cov_rank = 0;       // State::cov_rank
    int cov_taps = 0;           // State::cov_taps | State::taps_contig << 1 (diagonal Rhh: the tap-domain forms)
    int cov_path = 0;           // wce_debug_set_cov_path: 0 auto, 1 dense, 2 low-rank
    bool cm_on = false;         // State::cm_on: a constant-modulus operator is loaded (wce_ctx_set_modulus)
    bool cm_use = true;         // wce_debug_set_cm: A/B switch of that path
    std::vector<wce_complex> rhh;   // WCE_MMSE_COV ctx built here: the caller's Rhh (for wce_ctx_set_modulus)
    // Workspaces (FRAME_COV factors, MATLAB per-block rows), one per stream:
    // calls on different streams never share scratch, so they may run
    // concurrently (SURVEY 8(b) threading).  A call holds its stream's entry
    // locked from sizing to the last launch; plans own their workspace.
    std::mutex ws_mu;
    std::map<void *, std::unique_ptr<wce::Workspace>> ws_by_stream;
    int64_t ws_hint = 0;        // wce_ctx_reserve: minimum size of new entries
};

static constexpr int64_t WS_LD = 64;   // row stride (complex) of the workspace vectors
// workspace arrays of [frames][WS_LD] complex: h | u | w | (unused) | aux
// (per-block MMSE dots; the constant-modulus flags).  FRAME_COV uses h, u, w
// (REF in C semantics none: ref_fc_kernel writes H directly); MATLAB block
// averaging without FRAME_COV uses arrays 0..3 as the per-block W rows
// [frames * 4][WS_LD].
static constexpr int64_t WS_ARRAYS = 5;

static thread_local std::string g_err;

static int fail(int code, const char *what)
{
    g_err = what;
    return code;
}

static int hipfail(hipError_t e, const char *what)
{
    g_err = std::string(what) + ": " + hipGetErrorString(e);
    return WCE_EHIP;
}

#define HIPCHECK(x, what)                         \
    do {                                          \
        hipError_t e_ = (x);                      \
        if (e_ != hipSuccess) return hipfail(e_, what); \
    } while (0)

static int check_device(int device)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return fail(WCE_ENODEV, "no HIP device");
    if (device < 0 || device >= n) return fail(WCE_EINVAL, "device index out of range");
    hipDeviceProp_t prop;
    HIPCHECK(hipGetDeviceProperties(&prop, device), "hipGetDeviceProperties");
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return fail(WCE_ENODEV, "libwce is built for gfx950 (MI355X) only");
    return WCE_OK;
}

namespace {
struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int d)
    {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != d) (void)hipSetDevice(d);
    }
    ~DeviceGuard()
    {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};
}  // namespace

extern "C" {

const char *wce_last_error(void) { return g_err.c_str(); }
const char *wce_version(void) { return "wce 0.1.0 (gfx950)"; }

int wce_ctx_create_empty(wce_ctx **out, int device)
{
    if (!out) return fail(WCE_EINVAL, "null ctx pointer");
    int rc = check_device(device);
    if (rc) return rc;
    wce_ctx *c = new (std::nothrow) wce_ctx();
    if (!c) return fail(WCE_ENOMEM, "ctx alloc");
    c->device = device;
    DeviceGuard g(device);
    hipError_t e = hipMalloc(&c->d_state, sizeof(State));
    if (e != hipSuccess) { delete c; return hipfail(e, "hipMalloc(state)"); }
    e = hipMemset(c->d_state, 0, sizeof(State));
    if (e != hipSuccess) { (void)hipFree(c->d_state); delete c; return hipfail(e, "hipMemset(state)"); }
    *out = c;
    return WCE_OK;
}

int wce_ctx_create(wce_ctx **out, int device, const wce_complex *tx_pre, const wce_complex *rx_pre, double ow2,
                   int mode)
{
    if (!out || !tx_pre || !rx_pre) return fail(WCE_EINVAL, "null argument");
    if (mode != WCE_MMSE_REF && mode != WCE_MMSE_TEXTBOOK) return fail(WCE_EINVAL, "bad mmse mode");
    if (!(ow2 > 0)) return fail(WCE_EINVAL, "ow2 must be > 0");
    wce_ctx *c = nullptr;
    int rc = wce_ctx_create_empty(&c, device);
    if (rc) return rc;
    wce::ldc txl[wce::NSC], rxl[wce::NSC], hlt[wce::NSC];
    for (int k = 0; k < wce::NSC; k++) {
        txl[k].re = tx_pre[k].re; txl[k].im = tx_pre[k].im;
        rxl[k].re = rx_pre[k].re; rxl[k].im = rx_pre[k].im;
    }
    wce::host_lt_ls(txl, rxl, hlt);
    rc = wce::host_build_state(&c->host, wce::host_reference_F(), wce::host_reference_invF(), hlt, txl, ow2, mode);
    if (rc) { wce_ctx_destroy(c); return fail(rc, "state build"); }
    c->has_host = true;
    c->mode = mode;
    DeviceGuard g(device);
    hipError_t e = hipMemcpy(c->d_state, &c->host, sizeof(State), hipMemcpyHostToDevice);
    if (e != hipSuccess) { wce_ctx_destroy(c); return hipfail(e, "upload state"); }
    c->ready = true;
    *out = c;
    return WCE_OK;
}

int wce_ctx_create_cov(wce_ctx **out, int device, const wce_complex *tx_pre, const wce_complex *rx_pre,
                       const wce_complex *Rhh, double ow2)
{
    if (!out || !tx_pre || !rx_pre || !Rhh) return fail(WCE_EINVAL, "null argument");
    if (!(ow2 > 0)) return fail(WCE_EINVAL, "ow2 must be > 0");
    State *h = new (std::nothrow) State;
    if (!h) return fail(WCE_ENOMEM, "alloc");
    int rc = wce_state_build_cov(h, sizeof(State), tx_pre, rx_pre, Rhh, ow2);
    if (rc) { delete h; return fail(rc, "covariance state build"); }
    wce_ctx *c = nullptr;
    rc = wce_ctx_create_empty(&c, device);
    if (rc) { delete h; return rc; }
    rc = wce_ctx_load_state(c, h, sizeof(State));
    if (!rc) {
        c->host = *h;
        c->has_host = true;
        c->rhh.assign(Rhh, Rhh + wce::NSC * wce::NSC);
    }
    delete h;
    if (rc) { wce_ctx_destroy(c); return rc; }
    *out = c;
    return WCE_OK;
}

int wce_ctx_destroy(wce_ctx *c)
{
    if (!c) return WCE_OK;
    {
        DeviceGuard g(c->device);
        if (c->d_state) (void)hipFree(c->d_state);
        for (auto &kv : c->ws_by_stream)
            if (kv.second->p) (void)hipFree(kv.second->p);
    }
    delete c;
    return WCE_OK;
}

int wce_ctx_state(wce_ctx *c, void **ptr, size_t *bytes)
{
    if (!c) return fail(WCE_EINVAL, "null ctx");
    if (ptr) *ptr = c->d_state;
    if (bytes) *bytes = sizeof(State);
    return WCE_OK;
}

int wce_ctx_mark_ready(wce_ctx *c)
{
    if (!c) return fail(WCE_EINVAL, "null ctx");
    DeviceGuard g(c->device);
    HIPCHECK(hipDeviceSynchronize(), "sync");
    std::unique_ptr<State> h(new (std::nothrow) State);
    if (!h) return fail(WCE_ENOMEM, "alloc");
    HIPCHECK(hipMemcpy(h.get(), c->d_state, sizeof(State), hipMemcpyDeviceToHost), "read state");
    if (!wce::state_ok(h.get()))
        return fail(WCE_ESTATE, "state buffer does not hold a valid state of this build (magic, layout, size, mode, rank)");
    // the host copy (wce_ctx_set_modulus rebuilds from it) stays only if the
    // device now holds exactly it; another state drops it
    if (c->has_host && std::memcmp(h.get(), &c->host, sizeof(State)) != 0) {
        c->has_host = false;
        c->rhh.clear();
    }
    c->mode = h->mode;
    c->cov_rank = h->cov_rank;
    c->cov_k0 = h->cov_k0;
    c->cov_taps = (h->cov_taps ? 1 : 0) | (h->taps_contig ? 2 : 0);
    c->cm_on = h->cm_on != 0;
    c->ready = true;
    return WCE_OK;
}

int wce_ctx_load_state(wce_ctx *c, const void *host_state, size_t bytes)
{
    if (!c || !host_state || bytes < sizeof(State)) return fail(WCE_EINVAL, "bad state blob");
    const State *st = static_cast<const State *>(host_state);
    if (!wce::state_ok(st))
        return fail(WCE_ESTATE, "state blob is not a valid state of this build (magic, layout, size, mode, rank)");
    DeviceGuard g(c->device);
    HIPCHECK(hipMemcpy(c->d_state, host_state, sizeof(State), hipMemcpyHostToDevice), "upload state");
    if (c->has_host && std::memcmp(st, &c->host, sizeof(State)) != 0) {   // see wce_ctx_mark_ready
        c->has_host = false;
        c->rhh.clear();
    }
    c->mode = st->mode;
    c->cov_k0 = st->cov_k0;
    c->cov_rank = st->cov_rank;
    c->cov_taps = (st->cov_taps ? 1 : 0) | (st->taps_contig ? 2 : 0);
    c->cm_on = st->cm_on != 0;
    c->ready = true;
    return WCE_OK;
}

int wce_ctx_get_shared(wce_ctx *c, wce_complex *h_lt, wce_complex *C, double *a, double *b)
{
    if (!c) return fail(WCE_EINVAL, "null ctx");
    if (!c->ready) return fail(WCE_ESTATE, "ctx not ready");
    State *h = new (std::nothrow) State;
    if (!h) return fail(WCE_ENOMEM, "alloc");
    DeviceGuard g(c->device);
    hipError_t e = hipMemcpy(h, c->d_state, sizeof(State), hipMemcpyDeviceToHost);
    if (e != hipSuccess) { delete h; return hipfail(e, "download state"); }
    if (h_lt) std::memcpy(h_lt, h->h_lt, sizeof(wce_complex) * wce::NSC);
    if (C)
        for (int i = 0; i < wce::NSC; i++)
            std::memcpy(C + i * wce::NSC, h->C + 2 * i * wce::CLD, sizeof(wce_complex) * wce::NSC);
    if (a) *a = h->acoef;
    if (b) *b = h->bcoef;
    delete h;
    return WCE_OK;
}

// the WCE_MMSE_COV solve this ctx runs: -1 dense Ryy solve, else the block
// row of the embedded Gram system (mmse_lr_kernel)
static int cov_lr_k0(const wce_ctx *c)
{
    if (c->mode != WCE_MMSE_COV) return -1;
    if (c->cov_path == 1) return -1;
    if (c->cov_path == 2) {
        const int k0 = (wce::NSC - c->cov_rank) / 8;
        return k0 < wce::COV_K0_MAX ? k0 : wce::COV_K0_MAX;
    }
    return c->cov_k0;
}

int wce_ctx_cov_info(wce_ctx *c, int *rank, int *low_rank, double *lambda_max, double *lambda_min)
{
    if (!c) return fail(WCE_EINVAL, "null ctx");
    if (!c->ready) return fail(WCE_ESTATE, "ctx not ready");
    if (c->mode != WCE_MMSE_COV) return fail(WCE_EINVAL, "not a WCE_MMSE_COV context");
    double lm[2] = {0.0, 0.0};
    DeviceGuard g(c->device);
    HIPCHECK(hipMemcpy(lm, reinterpret_cast<char *>(c->d_state) + offsetof(State, cov_lmax), sizeof(lm),
                       hipMemcpyDeviceToHost), "read state eigenvalues");
    if (rank) *rank = c->cov_rank;
    if (low_rank) *low_rank = cov_lr_k0(c) >= 0;
    if (lambda_max) *lambda_max = lm[0];
    if (lambda_min) *lambda_min = lm[1];
    return WCE_OK;
}

int wce_ctx_set_modulus(wce_ctx *c, const wce_complex *x_ref)
{
    if (!c) return fail(WCE_EINVAL, "null ctx");
    if (!c->ready) return fail(WCE_ESTATE, "ctx not ready");
    if (c->mode != WCE_MMSE_COV) return fail(WCE_EINVAL, "wce_ctx_set_modulus: not a WCE_MMSE_COV context");
    if (!c->has_host || c->rhh.empty())
        return fail(WCE_ESTATE, "wce_ctx_set_modulus needs the ctx that built the state (wce_ctx_create_cov); "
                                "set it before the broadcast, or use wce_state_set_modulus on the blob");
    int rc = wce::host_build_cm(&c->host, wce::host_reference_F(), c->rhh.data(), x_ref);
    if (rc) return fail(rc, "constant-modulus operator: x_ref not finite, or Rhh / state mismatch");
    DeviceGuard g(c->device);
    HIPCHECK(hipDeviceSynchronize(), "sync before state update");   // no estimate may read the old state mid-copy
    HIPCHECK(hipMemcpy(c->d_state, &c->host, sizeof(State), hipMemcpyHostToDevice), "upload state");
    c->cm_on = c->host.cm_on != 0;
    return WCE_OK;
}

extern "C" int wce_debug_set_cm(wce_ctx *c, int on)
{
    if (!c) return fail(WCE_EINVAL, "null ctx");
    c->cm_use = on != 0;
    return WCE_OK;
}

extern "C" int wce_debug_set_cov_path(wce_ctx *c, int path)
{
    if (!c) return fail(WCE_EINVAL, "null ctx");
    if (path < 0 || path > 2) return fail(WCE_EINVAL, "cov path: 0 auto, 1 dense, 2 low-rank");
    c->cov_path = path;
    return WCE_OK;
}

extern "C" const char *wce_debug_lr_kernel(wce_ctx *c, long long units)
{
    if (!c || !c->ready || c->mode != WCE_MMSE_COV) return "";
    const int k0 = cov_lr_k0(c);
    if (k0 < 0) return "";
    DeviceGuard g(c->device);   // cu_count() reads the current device
    return wce::lr_kernel_name(k0, c->cov_rank, c->cov_taps, units);
}

static int check_frames(const wce_frames *in, bool need_blocks)
{
    if (!in) return fail(WCE_EINVAL, "null frames");
    if (in->n_frames < 0) return fail(WCE_EINVAL, "n_frames < 0");
    if (in->n_frames == 0) return WCE_OK;
    if (in->n_frames > INT32_MAX) return fail(WCE_EINVAL, "n_frames > 2^31 - 1 (one wave per frame in a 1-D grid)");
    if (!in->tx || !in->rx) return fail(WCE_EINVAL, "tx/rx required");
    if (in->block < 0 || in->block >= wce::NBLK) return fail(WCE_EINVAL, "block out of range");
    if (in->semantics != WCE_SEM_C && in->semantics != WCE_SEM_MATLAB) return fail(WCE_EINVAL, "bad semantics");
    if (in->semantics == WCE_SEM_MATLAB && in->n_frames > 0 && in->block_stride < wce::NSC)
        return fail(WCE_EINVAL, "MATLAB semantics reads blocks 0..3: block_stride < 53");
    if (in->block_stride < wce::NSC && (need_blocks || in->block > 0))
        return fail(WCE_EINVAL, "block_stride < 53");
    const int last = need_blocks ? wce::NBLK - 1 : (in->semantics == WCE_SEM_MATLAB ? 3 : in->block);
    const int64_t span = (int64_t)last * in->block_stride + wce::NSC;
    if (in->n_frames > 1 && in->frame_stride < span) return fail(WCE_EINVAL, "frame_stride too small");
    if (in->rx_pre && in->n_frames > 1 && in->pre_stride < wce::NSC) return fail(WCE_EINVAL, "pre_stride < 53");
    return WCE_OK;
}

static wce::LsArgs ls_args(const wce_frames *in, const wce_outputs *out, uint32_t mask, uint32_t eq_src)
{
    wce::LsArgs a{};
    a.tx = reinterpret_cast<const double *>(in->tx);
    a.rx = reinterpret_cast<const double *>(in->rx);
    a.rx_pre = reinterpret_cast<const double *>(in->rx_pre);
    a.tx_pre = reinterpret_cast<const double *>(in->tx_pre);
    a.fs = in->frame_stride; a.bs = in->block_stride; a.ps = in->pre_stride; a.n = in->n_frames; a.blk = in->block;
    a.matlab = in->semantics == WCE_SEM_MATLAB;
    a.mask = mask & (WCE_EST_LS_ALL | WCE_EQUALIZE);
    a.lt = reinterpret_cast<double *>(out->lt_ls);
    a.lin = reinterpret_cast<double *>(out->ps_linear);
    a.cub = reinterpret_cast<double *>(out->ps_cubic);
    a.snc = reinterpret_cast<double *>(out->ps_sinc);
    a.eq = reinterpret_cast<double *>(out->eq);
    a.os = out->out_stride; a.eqfs = out->eq_frame_stride; a.eqbs = out->eq_block_stride;
    a.eq_src = eq_src;
    a.f32 = (out->flags & WCE_OUT_LS_F32) != 0;
    if (a.mask & WCE_EQUALIZE) a.mask |= eq_src;   // the blend needs that PS estimate
    return a;
}

static wce::SolveArgs solve_args(const wce_ctx *c, const wce_frames *in, wce_complex *W, int64_t w_stride)
{
    wce::SolveArgs a{};
    if (c->mode == WCE_MMSE_TEXTBOOK) {   // C = c c': Ryy built from the shared vector
        a.cu = c->d_state->cvec;
        a.cw = nullptr;
        a.cs = 0;
        a.hout = c->bdot;
    } else if (c->mode == WCE_MMSE_REF && c->bdot) {   // C_ref = u w^T (a = 0: no Ryy build)
        a.cu = c->d_state->cvec;
        a.cw = c->d_state->cwvec;
        a.cs = 0;
        a.hout = 1;
        a.ref_pilots = 1;   // Ryy = 2 ow2 I, X = pilots: s = w^T X rx / b from 4 subcarriers
    }
    a.tx = reinterpret_cast<const double *>(in->tx);
    a.rx = reinterpret_cast<const double *>(in->rx);
    a.fs = in->frame_stride; a.bs = in->block_stride; a.n = in->n_frames;
    const bool ml = in->semantics == WCE_SEM_MATLAB;
    a.blk = ml ? 0 : in->block;
    a.nblk = ml ? 4 : 1;
    a.w = reinterpret_cast<double *>(W);
    a.ws = w_stride;
    return a;
}

int wce_mmse_solve(wce_ctx *c, const wce_frames *in, wce_complex *W, int64_t w_stride, void *stream)
{
    if (!c) return fail(WCE_EINVAL, "null ctx");
    if (!c->ready) return fail(WCE_ESTATE, "ctx not ready");
    int rc = check_frames(in, false);
    if (rc) return rc;
    if (in->n_frames == 0) return WCE_OK;
    if (!W || (in->n_frames > 1 && w_stride < wce::NSC)) return fail(WCE_EINVAL, "bad W");
    if (in->semantics != WCE_SEM_C)
        return fail(WCE_EINVAL, "wce_mmse_solve (profiling entry) takes C semantics; MATLAB runs via wce_estimate");
    if (cov_lr_k0(c) >= 0)
        return fail(WCE_EINVAL, "wce_mmse_solve: this WCE_MMSE_COV ctx runs the low-rank path (H = U s, no W / apply "
                                "stages); use wce_estimate");
    wce::SolveArgs a = solve_args(c, in, W, w_stride);
    if (a.hout) {   // the profiling pair solve -> apply keeps W = X z: rank-1 build only
        a.hout = 0;
        if (c->mode != WCE_MMSE_TEXTBOOK) a.cu = a.cw = nullptr;
    }
    DeviceGuard g(c->device);
    rc = wce::launch_mmse_solve(c->d_state, a, stream);
    return rc ? fail(rc, "mmse_solve launch") : WCE_OK;
}

int wce_mmse_apply(wce_ctx *c, const wce_complex *W, wce_complex *H, int64_t stride, int64_t n, void *stream)
{
    if (!c) return fail(WCE_EINVAL, "null ctx");
    if (!c->ready) return fail(WCE_ESTATE, "ctx not ready");
    if (n < 0) return fail(WCE_EINVAL, "n < 0");
    if (n == 0) return WCE_OK;
    if (!W || !H || (n > 1 && stride < wce::NSC)) return fail(WCE_EINVAL, "bad W/H");
    DeviceGuard g(c->device);
    int rc = wce::launch_mmse_apply(c->d_state, reinterpret_cast<const double *>(W), reinterpret_cast<double *>(H),
                                    stride, n, stream);
    return rc ? fail(rc, "mmse_apply launch") : WCE_OK;
}

int wce_nonfinite_scan(wce_ctx *c, const void *H, int64_t stride, int64_t n, uint32_t flags, uint32_t *bitmap,
                       unsigned long long *n_bad, void *stream)
{
    if (!c) return fail(WCE_EINVAL, "null ctx");
    if (n < 0) return fail(WCE_EINVAL, "n < 0");
    if (flags & ~(uint32_t)WCE_OUT_LS_F32) return fail(WCE_EINVAL, "unknown flags");
    if (n == 0) return WCE_OK;
    if (!H || !bitmap || (n > 1 && stride < wce::NSC)) return fail(WCE_EINVAL, "bad H/bitmap/stride");
    DeviceGuard g(c->device);
    int rc = wce::launch_nonfinite_scan(reinterpret_cast<const double *>(H), stride, n, (flags & WCE_OUT_LS_F32) != 0,
                                        bitmap, n_bad, stream);
    return rc ? fail(rc, "nonfinite_scan launch") : WCE_OK;
}

// x87 long double complex <-> complex double (wce_ldconv.hip)
static int ldc_convert(const void *src, void *dst, int64_t n, bool to_complex, void *stream)
{
    if (n < 0) return fail(WCE_EINVAL, "n < 0");
    if (n == 0) return WCE_OK;
    if (n > (int64_t)0x7fffffff * 256) return fail(WCE_EINVAL, "n too large for one launch");   // also keeps n * 32 in range
    if (!src || !dst) return fail(WCE_EINVAL, "null src/dst");
    if ((reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst)) & 15)
        return fail(WCE_EINVAL, "src/dst not 16-byte aligned");   // 16-B vector loads and stores
    const char *a = static_cast<const char *>(src), *b = static_cast<const char *>(dst);
    const int64_t sb = n * (to_complex ? 32 : 16), db = n * (to_complex ? 16 : 32);
    if (a < b + db && b < a + sb) return fail(WCE_EINVAL, "src and dst overlap");
    const int rc = wce::launch_ldc_convert(src, dst, n, to_complex, stream);
    return rc ? fail(rc, "ldc convert launch") : WCE_OK;
}

extern "C" int wce_ldc_to_complex(const void *src, wce_complex *dst, int64_t n, void *stream)
{
    return ldc_convert(src, dst, n, true, stream);
}

extern "C" int wce_complex_to_ldc(const wce_complex *src, void *dst, int64_t n, void *stream)
{
    return ldc_convert(src, dst, n, false, stream);
}

// grow `w` to n frames; the old buffer may still be read by work queued on
// `stream`, so that stream drains first (hipFree would wait for it anyway)
static int grow_ws(wce_ctx *c, wce::Workspace &w, int64_t n, void *stream)
{
    if (n <= w.frames) return WCE_OK;
    DeviceGuard g(c->device);
    if (w.p) {
        HIPCHECK(hipStreamSynchronize((hipStream_t)stream), "sync before workspace growth");
        (void)hipFree(w.p);
        w.p = nullptr;
        w.frames = 0;
    }
    HIPCHECK(hipMalloc(&w.p, (size_t)n * WS_ARRAYS * WS_LD * 2 * sizeof(double)), "hipMalloc(workspace)");
    w.frames = n;
    return WCE_OK;
}

// stream's workspace entry (created on first use), returned LOCKED
static wce::Workspace *stream_ws(wce_ctx *c, void *stream, std::unique_lock<std::mutex> &lk)
{
    wce::Workspace *w;
    {
        std::lock_guard<std::mutex> g(c->ws_mu);
        auto &slot = c->ws_by_stream[stream];
        if (!slot) slot.reset(new (std::nothrow) wce::Workspace);
        w = slot.get();
    }
    if (w) lk = std::unique_lock<std::mutex>(w->mu);
    return w;
}

int wce_ctx_reserve_stream(wce_ctx *c, int64_t n, void *stream)
{
    if (!c) return fail(WCE_EINVAL, "null ctx");
    if (n < 0) return fail(WCE_EINVAL, "n_frames < 0");
    std::unique_lock<std::mutex> lk;
    wce::Workspace *w = stream_ws(c, stream, lk);
    if (!w) return fail(WCE_ENOMEM, "workspace entry");
    return grow_ws(c, *w, n, stream);
}

int wce_ctx_reserve(wce_ctx *c, int64_t n)
{
    if (!c) return fail(WCE_EINVAL, "null ctx");
    if (n < 0) return fail(WCE_EINVAL, "n_frames < 0");
    {
        std::lock_guard<std::mutex> g(c->ws_mu);
        if (n > c->ws_hint) c->ws_hint = n;
    }
    return wce_ctx_reserve_stream(c, n, nullptr);
}

// WCE_MMSE_FRAME_COV: H_LT_f -> factors u_f, w_f of C_f (MFMA matvec, and for
// REF the folded pilot-row map), into the solve arguments.  lt_ready: the
// caller's LT_LS output already holds H_LT.  REF in C semantics takes one
// launch (ref_fc_kernel) that writes H = u s itself and sets *done.
// REF in C semantics runs ref_fc_kernel: one launch, no workspace.  The fused
// LS epilogue after it must be ref_ls_elem_kernel (the default REF_LS form);
// the wave-per-frame form takes the general path.
static bool ref_fc_path(const wce_ctx *c, const wce_frames *in, const wce::SolveArgs &sa)
{
    return c->mode == WCE_MMSE_REF && sa.ref_pilots && in->semantics == WCE_SEM_C &&
           wce::variant_value(wce::WCE_VARIANT_REF_FC) == 0 && wce::variant_value(wce::WCE_VARIANT_REF_LS) == 0;
}

static int prep_frame_cov(wce_ctx *c, const wce_frames *in, const wce_outputs *out, bool lt_ready,
                          wce::SolveArgs &sa, double *ws, bool *done, void *stream)
{
    const int64_t n = in->n_frames;
    if (!in->rx_pre) return fail(WCE_EINVAL, "WCE_MMSE_FRAME_COV needs per-frame preambles (rx_pre)");
    int rc = WCE_OK;
    const State *st = c->d_state;
    *done = false;
    if (ref_fc_path(c, in, sa)) {
        rc = wce::launch_ref_fc(st, sa, reinterpret_cast<const double *>(in->rx_pre), in->pre_stride,
                                reinterpret_cast<const double *>(in->tx_pre), stream);
        if (rc) return fail(rc, "ref_fc launch (frame covariance)");
        *done = true;
        return WCE_OK;
    }
    if (!ws) return fail(WCE_EINVAL, "frame covariance workspace missing");
    double *hw = ws, *uw = hw + n * WS_LD * 2, *ww = uw + n * WS_LD * 2;
    if (c->mode == WCE_MMSE_TEXTBOOK && in->semantics == WCE_SEM_C && !lt_ready &&
        wce::variant_value(wce::WCE_VARIANT_REF_FC) == 0) {   // LT_LS and u = Mu h in one launch
        rc = wce::launch_fc_u(st, reinterpret_cast<const double *>(in->rx_pre), in->pre_stride,
                              reinterpret_cast<const double *>(in->tx_pre), uw, WS_LD, n, stream);
        if (rc) return fail(rc, "fc_u launch (frame covariance)");
        sa.cu = uw;
        sa.cw = nullptr;
        sa.cs = WS_LD;
        sa.hout = 1;
        return WCE_OK;
    }
    const double *h = hw;
    int64_t hs = WS_LD;
    if (lt_ready) {
        h = reinterpret_cast<const double *>(out->lt_ls);
        hs = out->out_stride;
    } else {
        wce::LsArgs a{};
        a.tx = reinterpret_cast<const double *>(in->tx);
        a.rx = reinterpret_cast<const double *>(in->rx);
        a.rx_pre = reinterpret_cast<const double *>(in->rx_pre);
        a.tx_pre = reinterpret_cast<const double *>(in->tx_pre);
        a.fs = in->frame_stride; a.bs = in->block_stride; a.ps = in->pre_stride; a.n = n; a.blk = in->block;
        a.matlab = in->semantics == WCE_SEM_MATLAB;
        a.mask = WCE_EST_LT_LS;
        a.lt = hw;
        a.os = WS_LD;
        rc = wce::launch_ls(c->d_state, a, stream);
        if (rc) return fail(rc, "ls launch (H_LT for frame covariance)");
    }
    rc = wce::launch_matvec(st->Mu, nullptr, h, hs, uw, nullptr, WS_LD, n, false, stream);   // u
    if (!rc && c->mode == WCE_MMSE_REF) rc = wce::launch_ref_w(st, h, hs, ww, WS_LD, n, stream);   // w, pilot rows
    if (rc) return fail(rc, "matvec launch (frame covariance)");
    sa.cu = uw;
    sa.cw = c->mode == WCE_MMSE_REF ? ww : nullptr;
    sa.cs = WS_LD;
    sa.hout = 1;
    return WCE_OK;
}

// fixed != nullptr: a plan's own workspace (capture time); otherwise the
// stream's entry, held locked until the last launch is queued
static int estimate_impl(wce_ctx *c, const wce_frames *in, const wce_outputs *out, uint32_t mask, void *stream,
                         wce::Workspace *fixed)
{
    if (!c || !out) return fail(WCE_EINVAL, "null argument");
    if (!c->ready) return fail(WCE_ESTATE, "ctx not ready");
    if (mask & ~0x7Fu) return fail(WCE_EINVAL, "unknown estimator bits");
    if ((mask & WCE_MMSE_FRAME_COV) && !(mask & WCE_EST_PS_MMSE))
        return fail(WCE_EINVAL, "WCE_MMSE_FRAME_COV modifies WCE_EST_PS_MMSE");
    const bool eq = (mask & WCE_EQUALIZE) != 0;
    int rc = check_frames(in, eq);
    if (rc) return rc;
    if (in->n_frames == 0 || mask == 0) return WCE_OK;
    const int64_t n = in->n_frames;
    if (n > 1 && out->out_stride < wce::NSC && (mask & 0x1F)) return fail(WCE_EINVAL, "out_stride < 53");
    if ((mask & WCE_EST_LT_LS) && !out->lt_ls) return fail(WCE_EINVAL, "lt_ls output missing");
    if ((mask & WCE_EST_PS_LINEAR) && !out->ps_linear) return fail(WCE_EINVAL, "ps_linear output missing");
    if ((mask & WCE_EST_PS_CUBIC) && !out->ps_cubic) return fail(WCE_EINVAL, "ps_cubic output missing");
    if ((mask & WCE_EST_PS_SINC) && !out->ps_sinc) return fail(WCE_EINVAL, "ps_sinc output missing");
    if ((mask & WCE_EST_PS_MMSE) && !out->ps_mmse) return fail(WCE_EINVAL, "ps_mmse output missing");
    if (out->flags & ~WCE_OUT_LS_F32) return fail(WCE_EINVAL, "unknown output flags");
    uint32_t eq_src = out->eq_source ? out->eq_source : WCE_EST_PS_LINEAR;
    if (eq) {
        if (!out->eq) return fail(WCE_EINVAL, "eq output missing");
        if (eq_src != WCE_EST_PS_LINEAR && eq_src != WCE_EST_PS_CUBIC && eq_src != WCE_EST_PS_SINC)
            return fail(WCE_EINVAL, "eq_source must be a PS interpolation estimator");
        if (out->eq_block_stride < wce::NSC ||
            (n > 1 && out->eq_frame_stride < (wce::NBLK - 1) * out->eq_block_stride + wce::NSC))
            return fail(WCE_EINVAL, "eq strides too small");
    }
    if ((mask & WCE_MMSE_FRAME_COV) && !in->rx_pre)
        return fail(WCE_EINVAL, "WCE_MMSE_FRAME_COV needs per-frame preambles (rx_pre)");
    DeviceGuard g(c->device);
    const bool ls = (mask & (WCE_EST_LS_ALL | WCE_EQUALIZE)) != 0;
    const bool mmse = (mask & WCE_EST_PS_MMSE) != 0;
    // Config-5 fusion: the LS family and equalization ride in the MMSE solve's
    // epilogue (C semantics); otherwise one HBM-streaming LS pass.
    const int lr_k0 = (mask & WCE_MMSE_FRAME_COV) ? -1 : cov_lr_k0(c);   // WCE_MMSE_COV low-rank path
    // constant-modulus frames on the shared operator K (wce_ctx_set_modulus), the
    // rest on the per-frame kernels, which skip the flagged frames.  Not for ranks
    // 1..8 (the lane kernels are already bound by the frames' HBM traffic).
    const bool cm = mmse && c->mode == WCE_MMSE_COV && c->cm_on && c->cm_use && in->semantics == WCE_SEM_C &&
                    !(mask & WCE_MMSE_FRAME_COV) && (lr_k0 < 0 || c->cov_rank > wce::LRL_RMAX);
    const bool fuse = c->fuse && ls && mmse && in->semantics == WCE_SEM_C && lr_k0 < 0 && !cm;
    const wce::LsArgs la = ls_args(in, out, mask, eq_src);
    if (ls && !fuse) {
        rc = wce::launch_ls(c->d_state, la, stream);
        if (rc) return fail(rc, "ls launch");
    }
    if (!mmse) return WCE_OK;
    wce::SolveArgs sa = solve_args(c, in, out->ps_mmse, out->out_stride);
    const bool fc = (mask & WCE_MMSE_FRAME_COV) != 0;
    const bool split = sa.nblk > 1;   // MATLAB: one wave per (frame, block), averaged after
    if (split && n * sa.nblk > INT32_MAX) return fail(WCE_EINVAL, "n_frames * 4 > 2^31 - 1 (MATLAB semantics)");
    std::unique_lock<std::mutex> lk;
    double *ws = nullptr;
    if ((fc && !ref_fc_path(c, in, sa)) || split || cm) {
        wce::Workspace *w = fixed;
        if (!w) {
            w = stream_ws(c, stream, lk);
            if (!w) return fail(WCE_ENOMEM, "workspace entry");
            int64_t want = n;
            {
                std::lock_guard<std::mutex> hg(c->ws_mu);
                if (c->ws_hint > want) want = c->ws_hint;
            }
            rc = grow_ws(c, *w, want, stream);
            if (rc) return rc;
        } else if (w->frames < n) {
            return fail(WCE_EINVAL, "plan workspace too small");
        }
        ws = w->p;
    }
    if (fc) {
        const bool lt_ready = !fuse && (mask & WCE_EST_LT_LS) && !(out->flags & WCE_OUT_LS_F32);
        bool done = false;   // REF, C semantics: H written by the factor launch itself
        rc = prep_frame_cov(c, in, out, lt_ready, sa, ws, &done, stream);
        if (rc) return rc;
        if (done && !fuse) return WCE_OK;
        if (done) {   // the LS family + equalization still ride the one-element-per-thread pass
            sa.mmse_done = 1;
            rc = wce::launch_mmse_solve_ls(c->d_state, sa, la, stream);
            return rc ? fail(rc, "ls epilogue launch") : WCE_OK;
        }
    }
    double *aux = ws ? ws + (WS_ARRAYS - 1) * n * WS_LD * 2 : nullptr;
    if (split) {
        sa.split = 1;
        if (sa.hout) {
            sa.dots = aux;
        } else {
            sa.w = ws;
            sa.ws = WS_LD;
        }
    }
    double *H = reinterpret_cast<double *>(out->ps_mmse);
    if (cm) {   // flags (one byte per frame) in the aux array, unused in C semantics
        uint8_t *flags = reinterpret_cast<uint8_t *>(aux);
        rc = wce::launch_cm(c->d_state, sa, flags, stream);
        if (rc) return fail(rc, "constant-modulus launch");
        sa.skip = flags;
    }
    if (lr_k0 >= 0) {   // H = U s straight from the solve (split: H_b rows, then the block mean)
        rc = wce::launch_mmse_lr(c->d_state, lr_k0, c->cov_rank, c->cov_taps, sa, stream);
        if (rc) return fail(rc, "mmse_lr launch");
        if (split) rc = wce::launch_avg_blocks(ws, WS_LD, H, out->out_stride, n, stream);
        return rc ? fail(rc, "block average launch") : WCE_OK;
    }
    rc = fuse ? wce::launch_mmse_solve_ls(c->d_state, sa, la, stream) : wce::launch_mmse_solve(c->d_state, sa, stream);
    if (rc) return fail(rc, "mmse_solve launch");
    if (sa.hout && split) rc = wce::launch_fc_finish(sa, aux, H, out->out_stride, stream);
    else if (split) rc = wce::launch_matvec_avg(c->d_state->C, ws, WS_LD, sa.nblk, H, out->out_stride, n, stream);
    else if (!sa.hout) rc = wce::launch_mmse_apply(c->d_state, H, H, out->out_stride, n, stream, sa.skip);   // H = C W in place
    if (rc) return fail(rc, "mmse apply launch");
    return WCE_OK;
}

int wce_estimate(wce_ctx *c, const wce_frames *in, const wce_outputs *out, uint32_t mask, void *stream)
{
    return estimate_impl(c, in, out, mask, stream, nullptr);
}

struct wce_plan {
    wce_plan() = default;
    wce_plan(const wce_plan &) = delete;
    wce_plan &operator=(const wce_plan &) = delete;
    int device = 0;
    wce::Workspace ws;   // the plan's own scratch: replays never share a stream's
    hipGraph_t graph = nullptr;
    hipGraphExec_t exec = nullptr;
};

int wce_plan_create(wce_plan **out_plan, wce_ctx *c, const wce_frames *in, const wce_outputs *out, uint32_t mask)
{
    if (!out_plan || !c || !in || !out) return fail(WCE_EINVAL, "null argument");
    if (!c->ready) return fail(WCE_ESTATE, "ctx not ready");
    DeviceGuard g(c->device);
    wce_plan *p = new (std::nothrow) wce_plan;
    if (!p) return fail(WCE_ENOMEM, "alloc");
    p->device = c->device;
    // size the plan's workspace now: nothing may allocate while the stream is captured
    if ((mask & WCE_MMSE_FRAME_COV) || (in->semantics == WCE_SEM_MATLAB && (mask & WCE_EST_PS_MMSE)) ||
        (c->mode == WCE_MMSE_COV && c->cm_on && (mask & WCE_EST_PS_MMSE))) {
        int rc = grow_ws(c, p->ws, in->n_frames > 0 ? in->n_frames : 1, nullptr);
        if (rc) { delete p; return rc; }
    }
    auto fail_plan = [&](int code) {
        if (p->ws.p) (void)hipFree(p->ws.p);
        delete p;
        return code;
    };
    hipStream_t cs = nullptr;
    hipError_t e = hipStreamCreateWithFlags(&cs, hipStreamNonBlocking);
    if (e != hipSuccess) return fail_plan(hipfail(e, "plan capture stream"));
    e = hipStreamBeginCapture(cs, hipStreamCaptureModeThreadLocal);
    if (e != hipSuccess) {
        (void)hipStreamDestroy(cs);
        return fail_plan(hipfail(e, "hipStreamBeginCapture"));
    }
    const int rc = estimate_impl(c, in, out, mask, cs, &p->ws);   // validates, then records the launches
    hipGraph_t graph = nullptr;
    e = hipStreamEndCapture(cs, &graph);
    (void)hipStreamDestroy(cs);
    if (rc) {
        if (graph) (void)hipGraphDestroy(graph);
        return fail_plan(rc);
    }
    if (e != hipSuccess) return fail_plan(hipfail(e, "hipStreamEndCapture"));
    p->graph = graph;
    e = hipGraphInstantiate(&p->exec, graph, nullptr, nullptr, 0);
    if (e != hipSuccess) {
        (void)hipGraphDestroy(graph);
        return fail_plan(hipfail(e, "hipGraphInstantiate"));
    }
    *out_plan = p;
    return WCE_OK;
}

int wce_plan_launch(wce_plan *p, void *stream)
{
    if (!p || !p->exec) return fail(WCE_EINVAL, "null plan");
    DeviceGuard g(p->device);
    HIPCHECK(hipGraphLaunch(p->exec, (hipStream_t)stream), "hipGraphLaunch");
    return WCE_OK;
}

int wce_plan_destroy(wce_plan *p)
{
    if (!p) return WCE_OK;
    DeviceGuard g(p->device);
    if (p->exec) (void)hipGraphExecDestroy(p->exec);
    if (p->graph) (void)hipGraphDestroy(p->graph);
    if (p->ws.p) (void)hipFree(p->ws.p);
    delete p;
    return WCE_OK;
}

extern "C" int wce_debug_set_border_dot(wce_ctx *c, int on)
{
    if (!c) return fail(WCE_EINVAL, "null ctx");
    c->bdot = on != 0;
    return WCE_OK;
}

extern "C" int wce_debug_set_fusion(wce_ctx *c, int on)
{
    if (!c) return fail(WCE_EINVAL, "null ctx");
    c->fuse = on != 0;
    return WCE_OK;
}

int wce_synth_frames(wce_ctx *c, wce_complex *tx, wce_complex *rx, wce_complex *rx_pre, int64_t frame_stride,
                     int64_t block_stride, int64_t pre_stride, int64_t first_frame, int64_t n_frames, uint64_t seed,
                     const wce_complex *h_shared, double amplitude, double ow2, void *stream)
{
    if (!c) return fail(WCE_EINVAL, "null ctx");
    if (!c->ready) return fail(WCE_ESTATE, "ctx not ready");
    if (!rx || n_frames < 0 || first_frame < 0) return fail(WCE_EINVAL, "bad synth args");
    if (block_stride < wce::NSC || frame_stride < (wce::NBLK - 1) * block_stride + wce::NSC)
        return fail(WCE_EINVAL, "synth strides too small");
    if (rx_pre && pre_stride < wce::NSC) return fail(WCE_EINVAL, "pre_stride < 53");
    wce::SynthArgs a{};
    a.tx = reinterpret_cast<double *>(tx);
    a.rx = reinterpret_cast<double *>(rx);
    a.rx_pre = reinterpret_cast<double *>(rx_pre);
    a.fs = frame_stride; a.bs = block_stride; a.ps = pre_stride; a.first = first_frame; a.n = n_frames;
    a.seed = seed;
    a.h_shared = reinterpret_cast<const double *>(h_shared);
    a.amp = amplitude; a.ow2 = ow2;
    DeviceGuard g(c->device);
    int rc = wce::launch_synth(c->d_state, a, stream);
    return rc ? fail(rc, "synth launch") : WCE_OK;
}

// ---------------------------------------------------------------- front end
int wce_front_end_blocks(wce_ctx *c, const wce_complex *samples, int64_t packet_stride, int64_t n_frames,
                         int32_t n_blocks, wce_complex *sym, int64_t frame_stride, int64_t block_stride,
                         void *stream)
{
    if (!c) return fail(WCE_EINVAL, "null ctx");
    if (n_frames < 0 || n_blocks < 1) return fail(WCE_EINVAL, "n_frames < 0 or n_blocks < 1");
    if (n_frames == 0) return WCE_OK;
    if (!samples || !sym) return fail(WCE_EINVAL, "null buffer");
    if (packet_stride < (int64_t)n_blocks * WCE_SAMPLES_PER_BLOCK) return fail(WCE_EINVAL, "packet_stride < 80 n_blocks");
    if (block_stride < wce::NSC || frame_stride < (int64_t)(n_blocks - 1) * block_stride + wce::NSC)
        return fail(WCE_EINVAL, "output strides too small");
    if (n_frames * n_blocks >= (int64_t)1 << 31) return fail(WCE_EINVAL, "n_frames * n_blocks >= 2^31");
    wce::FrontArgs a{};
    a.src = reinterpret_cast<const double *>(samples);
    a.dst = reinterpret_cast<double *>(sym);
    a.ps = packet_stride; a.off = WCE_SAMPLES_PER_BLOCK - WCE_FFT_SIZE; a.fs = frame_stride; a.bs = block_stride;
    a.n_units = (uint32_t)(n_frames * n_blocks); a.nb = (uint32_t)n_blocks;
    DeviceGuard g(c->device);
    int rc = wce::launch_front(a, false, stream);
    return rc ? fail(rc, "front end launch") : WCE_OK;
}

int wce_front_end_preamble(wce_ctx *c, const wce_complex *lptot, int64_t lptot_stride, int64_t lptot_len,
                           int64_t n_frames, wce_complex *pre_fft, int64_t pre_stride, double *ow2, void *stream)
{
    if (!c) return fail(WCE_EINVAL, "null ctx");
    if (n_frames < 0) return fail(WCE_EINVAL, "n_frames < 0");
    if (n_frames == 0) return WCE_OK;
    if (!lptot || !pre_fft) return fail(WCE_EINVAL, "null buffer");
    if (lptot_len < 2 * WCE_FFT_SIZE || lptot_stride < lptot_len) return fail(WCE_EINVAL, "lptot_len < 128 or stride < len");
    if (pre_stride < wce::NSC) return fail(WCE_EINVAL, "pre_stride < 53");
    if (n_frames >= (int64_t)1 << 31) return fail(WCE_EINVAL, "n_frames >= 2^31");
    wce::FrontArgs a{};
    a.src = reinterpret_cast<const double *>(lptot);
    a.dst = reinterpret_cast<double *>(pre_fft);
    a.ow2 = ow2;
    a.ps = lptot_stride; a.off = lptot_len - 2 * WCE_FFT_SIZE; a.fs = pre_stride; a.bs = 0;
    a.n_units = (uint32_t)n_frames; a.nb = 1;
    DeviceGuard g(c->device);
    int rc = wce::launch_front(a, true, stream);
    return rc ? fail(rc, "front end launch") : WCE_OK;
}

// ---------------------------------------------------------------- runtime helpers
int wce_device_count(int *count)
{
    if (!count) return fail(WCE_EINVAL, "null");
    int n = 0;
    hipError_t e = hipGetDeviceCount(&n);
    *count = (e == hipSuccess) ? n : 0;
    return WCE_OK;
}
int wce_set_device(int d) { HIPCHECK(hipSetDevice(d), "hipSetDevice"); return WCE_OK; }
int wce_malloc(void **p, size_t bytes) { HIPCHECK(hipMalloc(p, bytes), "hipMalloc"); return WCE_OK; }
int wce_free(void *p) { HIPCHECK(hipFree(p), "hipFree"); return WCE_OK; }
int wce_memcpy_htod(void *d, const void *s, size_t b) { HIPCHECK(hipMemcpy(d, s, b, hipMemcpyHostToDevice), "htod"); return WCE_OK; }
int wce_memcpy_dtoh(void *d, const void *s, size_t b) { HIPCHECK(hipMemcpy(d, s, b, hipMemcpyDeviceToHost), "dtoh"); return WCE_OK; }
int wce_memcpy_dtod(void *d, const void *s, size_t b, void *st)
{
    HIPCHECK(hipMemcpyAsync(d, s, b, hipMemcpyDeviceToDevice, (hipStream_t)st), "dtod");
    return WCE_OK;
}
int wce_memset(void *d, int v, size_t b) { HIPCHECK(hipMemset(d, v, b), "hipMemset"); return WCE_OK; }
int wce_host_alloc(void **p, size_t b)
{
    if (!p) return fail(WCE_EINVAL, "null pointer");
    HIPCHECK(hipHostMalloc(p, b, hipHostMallocDefault), "hipHostMalloc");
    return WCE_OK;
}
int wce_host_free(void *p) { HIPCHECK(hipHostFree(p), "hipHostFree"); return WCE_OK; }
int wce_memcpy_htod_async(void *d, const void *s, size_t b, void *st)
{
    HIPCHECK(hipMemcpyAsync(d, s, b, hipMemcpyHostToDevice, (hipStream_t)st), "htod async");
    return WCE_OK;
}
int wce_memcpy_dtoh_async(void *d, const void *s, size_t b, void *st)
{
    HIPCHECK(hipMemcpyAsync(d, s, b, hipMemcpyDeviceToHost, (hipStream_t)st), "dtoh async");
    return WCE_OK;
}
int wce_stream_create(void **s)
{
    hipStream_t st;
    HIPCHECK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "hipStreamCreate");
    *s = st;
    return WCE_OK;
}
int wce_stream_destroy(void *s) { HIPCHECK(hipStreamDestroy((hipStream_t)s), "hipStreamDestroy"); return WCE_OK; }
int wce_stream_synchronize(void *s) { HIPCHECK(hipStreamSynchronize((hipStream_t)s), "hipStreamSynchronize"); return WCE_OK; }
int wce_event_create(void **ev)
{
    hipEvent_t e;
    HIPCHECK(hipEventCreate(&e), "hipEventCreate");
    *ev = e;
    return WCE_OK;
}
int wce_event_destroy(void *ev) { HIPCHECK(hipEventDestroy((hipEvent_t)ev), "hipEventDestroy"); return WCE_OK; }
int wce_event_record(void *ev, void *s) { HIPCHECK(hipEventRecord((hipEvent_t)ev, (hipStream_t)s), "hipEventRecord"); return WCE_OK; }
int wce_event_elapsed_ms(float *ms, void *a, void *b)
{
    HIPCHECK(hipEventSynchronize((hipEvent_t)b), "hipEventSynchronize");
    HIPCHECK(hipEventElapsedTime(ms, (hipEvent_t)a, (hipEvent_t)b), "hipEventElapsedTime");
    return WCE_OK;
}

}  // extern "C"

extern "C" int wce_debug_set_variant(int which, int value)
{
    const int rc = wce::set_variant(which, value);
    return rc ? fail(rc, "variant: which in [0, 5), value in [0, 16)") : WCE_OK;
}

extern "C" int wce_debug_set_flat_chunk(long long frames)
{
    const int rc = wce::set_flat_chunk(frames);
    return rc ? fail(rc, "flat chunk: 0, or a multiple of 32 in [32, 2^26]") : WCE_OK;
}

// ---- internal hooks for wce_multi.cpp (wce_internal.h)
namespace wce {
int api_fail(int code, const char *what) { return fail(code, what); }
int ctx_device(const wce_ctx *c) { return c ? c->device : -1; }
bool ctx_ready(const wce_ctx *c) { return c && c->ready; }
}  // namespace wce
