// wce_multi.cpp -- multi-GPU part of the C ABI (include/wce.h).
//
// Frames shard with no inter-GPU dependence; the one exchange is a broadcast
// of the packed shared state (wce::State) from the rank that built it, done
// in place in every rank's context buffer over RCCL (xGMI within a node).
// This replaces the reference's MPI_Bcast of F / Ryy (main_mpi.c:687-688,
// 727-728) and its rank-strided frame loops (main_mpi.c:99, 140).
//
// RCCL is dlopen'ed on first use (librccl.so.1): libwce has no link-time
// RCCL dependency, and inside a PyTorch process the soname resolves to the
// RCCL torch already loaded, so both share one RCCL and one HIP runtime.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>
#include <dlfcn.h>

#include <cstring>
#include <mutex>
#include <new>
#include <string>
#include <vector>

#include "wce_internal.h"

struct wce_comm {
    ncclComm_t nc = nullptr;
    int rank = 0, nranks = 1, device = 0;
    double *d_val = nullptr;   // 8-byte all-reduce buffer
};

namespace {

struct Rccl {
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) init_rank = nullptr;
    decltype(&ncclCommInitAll) init_all = nullptr;
    decltype(&ncclCommDestroy) destroy = nullptr;
    decltype(&ncclBroadcast) broadcast = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclGroupStart) group_start = nullptr;
    decltype(&ncclGroupEnd) group_end = nullptr;
    decltype(&ncclGetErrorString) error_string = nullptr;
    bool ok = false;
    std::string why;
};

const Rccl &rccl()
{
    static Rccl r;
    static std::once_flag once;
    std::call_once(once, [] {
        void *h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) {
            const char *e = dlerror();
            r.why = std::string("cannot load librccl.so.1: ") + (e ? e : "?");
            return;
        }
#define WCE_SYM(field, name)                                                  \
    r.field = reinterpret_cast<decltype(r.field)>(dlsym(h, name));            \
    if (!r.field) {                                                           \
        r.why = std::string("librccl.so.1 lacks ") + name;                    \
        return;                                                               \
    }
        WCE_SYM(get_unique_id, "ncclGetUniqueId")
        WCE_SYM(init_rank, "ncclCommInitRank")
        WCE_SYM(init_all, "ncclCommInitAll")
        WCE_SYM(destroy, "ncclCommDestroy")
        WCE_SYM(broadcast, "ncclBroadcast")
        WCE_SYM(all_reduce, "ncclAllReduce")
        WCE_SYM(group_start, "ncclGroupStart")
        WCE_SYM(group_end, "ncclGroupEnd")
        WCE_SYM(error_string, "ncclGetErrorString")
#undef WCE_SYM
        r.ok = true;
    });
    return r;
}

int nccl_fail(ncclResult_t e, const char *what)
{
    const Rccl &r = rccl();
    std::string m = std::string(what) + ": " + (r.error_string ? r.error_string(e) : "rccl error");
    return wce::api_fail(WCE_EHIP, m.c_str());
}

int hip_fail(hipError_t e, const char *what)
{
    std::string m = std::string(what) + ": " + hipGetErrorString(e);
    return wce::api_fail(WCE_EHIP, m.c_str());
}

// usable gfx950 device `d` (same checks as context creation)
int check_dev(int d)
{
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n == 0) return wce::api_fail(WCE_ENODEV, "no HIP device");
    if (d < 0 || d >= n) return wce::api_fail(WCE_EINVAL, "device index out of range");
    hipDeviceProp_t prop;
    hipError_t e = hipGetDeviceProperties(&prop, d);
    if (e != hipSuccess) return hip_fail(e, "hipGetDeviceProperties");
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return wce::api_fail(WCE_ENODEV, "libwce is built for gfx950 (MI355X) only");
    return WCE_OK;
}

struct DevGuard {
    int prev = -1;
    explicit DevGuard(int d)
    {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
        if (prev != d) (void)hipSetDevice(d);
    }
    ~DevGuard()
    {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

int rccl_ready()
{
    const Rccl &r = rccl();
    return r.ok ? WCE_OK : wce::api_fail(WCE_ENODEV, r.why.c_str());
}

int new_comm(wce_comm **out, ncclComm_t nc, int rank, int nranks, int device)
{
    wce_comm *c = new (std::nothrow) wce_comm();
    if (!c) return wce::api_fail(WCE_ENOMEM, "comm alloc");
    c->nc = nc;
    c->rank = rank;
    c->nranks = nranks;
    c->device = device;
    DevGuard g(device);
    hipError_t e = hipMalloc(&c->d_val, sizeof(double));
    if (e != hipSuccess) {
        rccl().destroy(nc);
        delete c;
        return hip_fail(e, "hipMalloc(comm scratch)");
    }
    *out = c;
    return WCE_OK;
}

// argument checks shared by the single and grouped broadcasts
int check_bcast(wce_ctx *ctx, const wce_comm *comm, int root)
{
    if (!ctx || !comm) return wce::api_fail(WCE_EINVAL, "null ctx or comm");
    if (root < 0 || root >= comm->nranks) return wce::api_fail(WCE_EINVAL, "root rank out of range");
    if (wce::ctx_device(ctx) != comm->device) return wce::api_fail(WCE_EINVAL, "ctx and comm are on different devices");
    if (comm->rank == root && !wce::ctx_ready(ctx))
        return wce::api_fail(WCE_ESTATE, "root context holds no valid state");
    return WCE_OK;
}

}  // namespace

extern "C" {

int wce_comm_unique_id(void *id)
{
    if (!id) return wce::api_fail(WCE_EINVAL, "null id");
    int rc = rccl_ready();
    if (rc) return rc;
    ncclUniqueId u;
    ncclResult_t e = rccl().get_unique_id(&u);
    if (e != ncclSuccess) return nccl_fail(e, "ncclGetUniqueId");
    static_assert(sizeof(u) == WCE_COMM_ID_BYTES, "unique id size");
    std::memcpy(id, &u, sizeof(u));
    return WCE_OK;
}

int wce_comm_init_rank(wce_comm **out, const void *id, int nranks, int rank, int device)
{
    if (!out || !id) return wce::api_fail(WCE_EINVAL, "null argument");
    if (nranks < 1 || rank < 0 || rank >= nranks) return wce::api_fail(WCE_EINVAL, "bad rank / nranks");
    int rc = check_dev(device);
    if (rc) return rc;
    rc = rccl_ready();
    if (rc) return rc;
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    ncclComm_t nc = nullptr;
    {
        DevGuard g(device);
        ncclResult_t e = rccl().init_rank(&nc, nranks, u, rank);
        if (e != ncclSuccess) return nccl_fail(e, "ncclCommInitRank");
    }
    return new_comm(out, nc, rank, nranks, device);
}

int wce_comm_init_all(wce_comm **comms, int ndev, const int *devices)
{
    if (!comms || !devices || ndev < 1) return wce::api_fail(WCE_EINVAL, "bad device list");
    for (int i = 0; i < ndev; ++i) {
        int rc = check_dev(devices[i]);
        if (rc) return rc;
        for (int j = 0; j < i; ++j)
            if (devices[j] == devices[i]) return wce::api_fail(WCE_EINVAL, "a device is listed twice");
    }
    int rc = rccl_ready();
    if (rc) return rc;
    std::vector<ncclComm_t> nc(ndev, nullptr);
    ncclResult_t e = rccl().init_all(nc.data(), ndev, devices);
    if (e != ncclSuccess) return nccl_fail(e, "ncclCommInitAll");
    for (int i = 0; i < ndev; ++i) {
        rc = new_comm(&comms[i], nc[i], i, ndev, devices[i]);
        if (rc) {
            for (int j = 0; j < i; ++j) wce_comm_destroy(comms[j]);
            for (int j = i + 1; j < ndev; ++j) rccl().destroy(nc[j]);
            return rc;
        }
    }
    return WCE_OK;
}

int wce_comm_destroy(wce_comm *c)
{
    if (!c) return WCE_OK;
    DevGuard g(c->device);
    if (c->d_val) (void)hipFree(c->d_val);
    ncclResult_t e = c->nc ? rccl().destroy(c->nc) : ncclSuccess;
    delete c;
    return e == ncclSuccess ? WCE_OK : nccl_fail(e, "ncclCommDestroy");
}

int wce_comm_info(const wce_comm *c, int *rank, int *nranks, int *device)
{
    if (!c) return wce::api_fail(WCE_EINVAL, "null comm");
    if (rank) *rank = c->rank;
    if (nranks) *nranks = c->nranks;
    if (device) *device = c->device;
    return WCE_OK;
}

int wce_ctx_broadcast_state(wce_ctx *ctx, wce_comm *comm, int root, void *stream)
{
    return wce_ctx_broadcast_state_all(&ctx, &comm, 1, root, &stream);
}

int wce_ctx_broadcast_state_all(wce_ctx **ctxs, wce_comm **comms, int n, int root, void **streams)
{
    if (!ctxs || !comms || n < 1) return wce::api_fail(WCE_EINVAL, "bad context list");
    for (int i = 0; i < n; ++i) {
        int rc = check_bcast(ctxs[i], comms[i], root);
        if (rc) return rc;
    }
    int rc = rccl_ready();
    if (rc) return rc;
    const Rccl &r = rccl();
    // one group: every rank's buffer is both send and receive (in place)
    ncclResult_t e = n > 1 ? r.group_start() : ncclSuccess;
    for (int i = 0; i < n && e == ncclSuccess; ++i) {
        void *ptr = nullptr;
        size_t bytes = 0;
        wce_ctx_state(ctxs[i], &ptr, &bytes);
        DevGuard g(comms[i]->device);
        e = r.broadcast(ptr, ptr, bytes, ncclUint8, root, comms[i]->nc, streams ? (hipStream_t)streams[i] : nullptr);
    }
    if (n > 1) {
        ncclResult_t e2 = r.group_end();
        if (e == ncclSuccess) e = e2;
    }
    if (e != ncclSuccess) return nccl_fail(e, "ncclBroadcast(state)");
    for (int i = 0; i < n; ++i) {
        DevGuard g(comms[i]->device);
        hipError_t he = hipStreamSynchronize(streams ? (hipStream_t)streams[i] : nullptr);
        if (he != hipSuccess) return hip_fail(he, "broadcast sync");
        rc = wce_ctx_mark_ready(ctxs[i]);   // validates the magic and caches the mode
        if (rc) return rc;
    }
    return WCE_OK;
}

int wce_comm_max_f64(wce_comm *comm, double *value, void *stream)
{
    return wce_comm_max_f64_all(&comm, 1, value, &stream);
}

int wce_comm_max_f64_all(wce_comm **comms, int n, double *values, void **streams)
{
    if (!comms || !values || n < 1) return wce::api_fail(WCE_EINVAL, "bad argument");
    for (int i = 0; i < n; ++i)
        if (!comms[i]) return wce::api_fail(WCE_EINVAL, "null comm");
    int rc = rccl_ready();
    if (rc) return rc;
    const Rccl &r = rccl();
    for (int i = 0; i < n; ++i) {
        DevGuard g(comms[i]->device);
        hipStream_t s = streams ? (hipStream_t)streams[i] : nullptr;
        hipError_t he = hipMemcpyAsync(comms[i]->d_val, &values[i], sizeof(double), hipMemcpyHostToDevice, s);
        if (he != hipSuccess) return hip_fail(he, "max: upload");
        he = hipStreamSynchronize(s);
        if (he != hipSuccess) return hip_fail(he, "max: upload sync");
    }
    ncclResult_t e = n > 1 ? r.group_start() : ncclSuccess;
    for (int i = 0; i < n && e == ncclSuccess; ++i) {
        DevGuard g(comms[i]->device);
        e = r.all_reduce(comms[i]->d_val, comms[i]->d_val, 1, ncclFloat64, ncclMax, comms[i]->nc,
                         streams ? (hipStream_t)streams[i] : nullptr);
    }
    if (n > 1) {
        ncclResult_t e2 = r.group_end();
        if (e == ncclSuccess) e = e2;
    }
    if (e != ncclSuccess) return nccl_fail(e, "ncclAllReduce(max)");
    for (int i = 0; i < n; ++i) {
        DevGuard g(comms[i]->device);
        hipStream_t s = streams ? (hipStream_t)streams[i] : nullptr;
        hipError_t he = hipMemcpyAsync(&values[i], comms[i]->d_val, sizeof(double), hipMemcpyDeviceToHost, s);
        if (he == hipSuccess) he = hipStreamSynchronize(s);
        if (he != hipSuccess) return hip_fail(he, "max: download");
    }
    return WCE_OK;
}

int wce_shard(int64_t total, int nranks, int rank, int64_t *first, int64_t *count)
{
    if (total < 0 || nranks < 1 || rank < 0 || rank >= nranks || !first || !count)
        return wce::api_fail(WCE_EINVAL, "bad shard arguments");
    const int64_t base = total / nranks, extra = total % nranks;
    *first = rank * base + (rank < extra ? rank : extra);
    *count = base + (rank < extra ? 1 : 0);
    return WCE_OK;
}

}  // extern "C"
