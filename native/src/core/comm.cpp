// Native RCCL tier: the inter-GPU transport of the slab decompositions (halo
// exchange between vertically adjacent slabs, global reductions), called
// directly from C instead of through torch.distributed's per-op Work/event
// machinery.
//
// Reference: the MPI tier the BASELINE north star describes (domain-decomposed
// halo exchange + global reductions; SURVEY.md §2 "MPI tier"), re-expressed as
// RCCL point-to-point and all-reduce over xGMI.
//
// Design
//   * ONE RCCL per process: the ncclXxx entry points are resolved with dlsym
//     from the librccl that torch already loaded (its path comes from Python),
//     so torch's process group and this communicator share one library and one
//     bootstrap implementation. The communicator itself is our own
//     (ncclCommInitRank with a unique id broadcast over torch.distributed).
//   * a halo exchange is one ncclGroupStart / {ncclSend, ncclRecv}* /
//     ncclGroupEnd on a dedicated non-blocking, highest-priority comm stream
//     (so its workgroups are dispatched ahead of the overlapped compute), forked from and
//     joined back into the caller's stream with two events:
//         start(stream): record ready@stream; comm waits ready; group p2p;
//                        record done@comm
//         wait(stream):  stream waits done
//     so everything the caller queues between start and wait (the interior
//     rows of a stencil) overlaps the xGMI transfer. Per step this costs the
//     RCCL group launch plus four HIP event calls — no Python objects.
//   * reductions (residual max, sums) run on the caller's stream directly.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>

#include "mpx/capi.h"
#include "../kernels/internal.hpp"

namespace mpx {
namespace {

struct RcclApi {
    decltype(&ncclGetUniqueId) GetUniqueId = nullptr;
    decltype(&ncclCommInitRank) CommInitRank = nullptr;
    decltype(&ncclCommDestroy) CommDestroy = nullptr;
    decltype(&ncclCommAbort) CommAbort = nullptr;
    decltype(&ncclCommGetAsyncError) CommGetAsyncError = nullptr;
    decltype(&ncclGetErrorString) GetErrorString = nullptr;
    decltype(&ncclGroupStart) GroupStart = nullptr;
    decltype(&ncclGroupEnd) GroupEnd = nullptr;
    decltype(&ncclSend) Send = nullptr;
    decltype(&ncclRecv) Recv = nullptr;
    decltype(&ncclAllReduce) AllReduce = nullptr;
    decltype(&ncclGetVersion) GetVersion = nullptr;
    decltype(&ncclCommCount) CommCount = nullptr;  // optional: world size as RCCL reports it
    void *handle = nullptr;
    std::string path;
};

RcclApi g_api;
std::mutex g_api_mu;

template <typename F>
bool bind(void *h, const char *name, F &fn) {
    fn = reinterpret_cast<F>(dlsym(h, name));
    return fn != nullptr;
}

struct Comm {
    ncclComm_t comm = nullptr;
    hipStream_t cstream = nullptr;
    hipEvent_t ready = nullptr, done = nullptr;
    int rank = 0, nranks = 1, device = 0;
    bool pending = false;  // a started exchange not yet joined
};

#define MPX_NCCL(call)                                                                           \
    do {                                                                                         \
        ncclResult_t r_ = (call);                                                                \
        if (r_ != ncclSuccess) {                                                                 \
            set_error("RCCL %s failed: %s", #call, g_api.GetErrorString ? g_api.GetErrorString(r_) : "?"); \
            return MPX_ERR_HIP;                                                                  \
        }                                                                                        \
    } while (0)

}  // namespace
}  // namespace mpx

using namespace mpx;

extern "C" int mpx_comm_load(const char *path) {
    std::lock_guard<std::mutex> lk(g_api_mu);
    if (g_api.handle) return MPX_OK;
    // RTLD_NOLOAD first: reuse the copy torch loaded, never a second RCCL
    void *h = path && *path ? dlopen(path, RTLD_NOW | RTLD_NOLOAD) : nullptr;
    if (!h && path && *path) h = dlopen(path, RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) {
        set_error("cannot load RCCL (%s): %s", path ? path : "", dlerror());
        return MPX_ERR_ARG;
    }
    RcclApi a;
    a.handle = h;
    bool ok = bind(h, "ncclGetUniqueId", a.GetUniqueId) && bind(h, "ncclCommInitRank", a.CommInitRank) &&
              bind(h, "ncclCommDestroy", a.CommDestroy) && bind(h, "ncclCommAbort", a.CommAbort) &&
              bind(h, "ncclCommGetAsyncError", a.CommGetAsyncError) &&
              bind(h, "ncclGetErrorString", a.GetErrorString) && bind(h, "ncclGroupStart", a.GroupStart) &&
              bind(h, "ncclGroupEnd", a.GroupEnd) && bind(h, "ncclSend", a.Send) && bind(h, "ncclRecv", a.Recv) &&
              bind(h, "ncclAllReduce", a.AllReduce) && bind(h, "ncclGetVersion", a.GetVersion);
    bind(h, "ncclCommCount", a.CommCount);
    if (!ok) {
        set_error("RCCL at %s lacks a required symbol", path ? path : "librccl.so.1");
        return MPX_ERR_ARG;
    }
    a.path = path ? path : "librccl.so.1";
    g_api = a;
    return MPX_OK;
}

extern "C" int mpx_comm_version(void) {
    int v = 0;
    if (!g_api.GetVersion || g_api.GetVersion(&v) != ncclSuccess) return -1;
    return v;
}

extern "C" int mpx_comm_unique_id(void *out, int nbytes) {
    MPX_CHECK_ARG(g_api.handle, "RCCL not loaded (mpx_comm_load)");
    MPX_CHECK_ARG(out && nbytes >= (int)sizeof(ncclUniqueId), "id buffer too small");
    ncclUniqueId id;
    MPX_NCCL(g_api.GetUniqueId(&id));
    std::memcpy(out, &id, sizeof(id));
    return (int)sizeof(id);
}

extern "C" int mpx_comm_init(void **out, int nranks, int rank, const void *id, int nbytes, int device) {
    MPX_CHECK_ARG(g_api.handle, "RCCL not loaded (mpx_comm_load)");
    MPX_CHECK_ARG(out && id && nbytes == (int)sizeof(ncclUniqueId), "bad unique id");
    MPX_CHECK_ARG(nranks >= 1 && rank >= 0 && rank < nranks, "bad rank");
    MPX_RETURN_IF_HIP_ERROR(hipSetDevice(device));
    Comm *c = new Comm();
    c->rank = rank;
    c->nranks = nranks;
    c->device = device;
    ncclUniqueId uid;
    std::memcpy(&uid, id, sizeof(uid));
    ncclResult_t r = g_api.CommInitRank(&c->comm, nranks, uid, rank);
    if (r != ncclSuccess) {
        set_error("ncclCommInitRank failed: %s", g_api.GetErrorString(r));
        delete c;
        return MPX_ERR_HIP;
    }
    // highest-priority comm stream: when a step's transfer and its interior
    // convolution become runnable together, the dispatcher places RCCL's few
    // workgroups first instead of queueing them behind thousands of conv waves
    int prio_lo = 0, prio_hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&prio_lo, &prio_hi);
    if (hipStreamCreateWithPriority(&c->cstream, hipStreamNonBlocking, prio_hi) != hipSuccess ||
        hipEventCreateWithFlags(&c->ready, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&c->done, hipEventDisableTiming) != hipSuccess) {
        set_error("comm stream/event creation failed");
        g_api.CommDestroy(c->comm);
        delete c;
        return MPX_ERR_HIP;
    }
    *out = c;
    return MPX_OK;
}

extern "C" int mpx_comm_destroy(void *h) {
    if (!h) return MPX_OK;
    Comm *c = static_cast<Comm *>(h);
    (void)hipSetDevice(c->device);
    if (c->cstream) (void)hipStreamSynchronize(c->cstream);
    if (c->comm) g_api.CommDestroy(c->comm);
    if (c->ready) (void)hipEventDestroy(c->ready);
    if (c->done) (void)hipEventDestroy(c->done);
    if (c->cstream) (void)hipStreamDestroy(c->cstream);
    delete c;
    return MPX_OK;
}

extern "C" int mpx_comm_rank(void *h) { return h ? static_cast<Comm *>(h)->rank : -1; }
extern "C" int mpx_comm_size(void *h) {
    if (!h) return -1;
    Comm *c = static_cast<Comm *>(h);
    int n = -1;
    if (g_api.CommCount && c->comm && g_api.CommCount(c->comm, &n) == ncclSuccess) return n;
    return c->nranks;
}

namespace {
int group_p2p(Comm *c, int n, const int *kind, void *const *ptr, const int64_t *bytes, const int *peer,
              hipStream_t s) {
    if (n == 0) return MPX_OK;
    MPX_NCCL(g_api.GroupStart());
    for (int i = 0; i < n; ++i) {
        if (peer[i] < 0 || peer[i] >= c->nranks || bytes[i] < 0) {
            g_api.GroupEnd();
            set_error("bad p2p op %d (peer %d, bytes %lld)", i, peer[i], (long long)bytes[i]);
            return MPX_ERR_ARG;
        }
        ncclResult_t r = kind[i] == 0 ? g_api.Send(ptr[i], (size_t)bytes[i], ncclUint8, peer[i], c->comm, s)
                                      : g_api.Recv(ptr[i], (size_t)bytes[i], ncclUint8, peer[i], c->comm, s);
        if (r != ncclSuccess) {
            g_api.GroupEnd();
            set_error("RCCL %s failed: %s", kind[i] == 0 ? "ncclSend" : "ncclRecv", g_api.GetErrorString(r));
            return MPX_ERR_HIP;
        }
    }
    MPX_NCCL(g_api.GroupEnd());
    return MPX_OK;
}
}  // namespace

// Grouped point-to-point in order on the caller's stream (no second queue).
// Measured on MI355X (profiles/comm_step.md): the RCCL kernel of a 4 x 32 KB
// exchange takes ~9 us alone but ~40 us when it shares the CUs with an
// overlapped 4096^2 convolution, and every cross-queue join adds a 7-16 us
// barrier-packet gap — so in-order exchange + one full-image launch beats the
// fork/join overlap for halos this small.
extern "C" int mpx_comm_p2p(void *h, int n, const int *kind, void *const *ptr, const int64_t *bytes,
                            const int *peer, void *stream) {
    MPX_CHECK_ARG(h, "null communicator");
    MPX_CHECK_ARG(n >= 0 && (n == 0 || (kind && ptr && bytes && peer)), "bad op list");
    return group_p2p(static_cast<Comm *>(h), n, kind, ptr, bytes, peer, as_stream(stream));
}

// Grouped point-to-point: op i sends (kind 0) or receives (kind 1) bytes[i]
// bytes at ptr[i] to / from rank peer[i]. Ordered after the work already
// queued on `stream`; the caller joins with mpx_comm_p2p_wait.
extern "C" int mpx_comm_p2p_start(void *h, int n, const int *kind, void *const *ptr, const int64_t *bytes,
                                  const int *peer, void *stream) {
    MPX_CHECK_ARG(h, "null communicator");
    Comm *c = static_cast<Comm *>(h);
    MPX_CHECK_ARG(!c->pending, "previous exchange not joined (mpx_comm_p2p_wait)");
    MPX_CHECK_ARG(n >= 0 && (n == 0 || (kind && ptr && bytes && peer)), "bad op list");
    hipStream_t s = as_stream(stream);
    MPX_RETURN_IF_HIP_ERROR(hipEventRecord(c->ready, s));
    MPX_RETURN_IF_HIP_ERROR(hipStreamWaitEvent(c->cstream, c->ready, 0));
    const int rc = group_p2p(c, n, kind, ptr, bytes, peer, c->cstream);
    if (rc != MPX_OK) return rc;
    MPX_RETURN_IF_HIP_ERROR(hipEventRecord(c->done, c->cstream));
    c->pending = true;
    return MPX_OK;
}

extern "C" int mpx_comm_p2p_wait(void *h, void *stream) {
    MPX_CHECK_ARG(h, "null communicator");
    Comm *c = static_cast<Comm *>(h);
    if (!c->pending) return MPX_OK;
    MPX_RETURN_IF_HIP_ERROR(hipStreamWaitEvent(as_stream(stream), c->done, 0));
    c->pending = false;
    return MPX_OK;
}

// dtype: 0 f64, 1 f32, 2 i32, 3 u64; op: 0 sum, 1 max, 2 min
extern "C" int mpx_comm_allreduce(void *h, const void *send, void *recv, int64_t count, int dtype, int op,
                                  void *stream) {
    MPX_CHECK_ARG(h, "null communicator");
    MPX_CHECK_ARG(count >= 0 && dtype >= 0 && dtype <= 3 && op >= 0 && op <= 2, "bad all-reduce arguments");
    static const ncclDataType_t dt[] = {ncclFloat64, ncclFloat32, ncclInt32, ncclUint64};
    static const ncclRedOp_t ro[] = {ncclSum, ncclMax, ncclMin};
    Comm *c = static_cast<Comm *>(h);
    MPX_NCCL(g_api.AllReduce(send, recv, (size_t)count, dt[dtype], ro[op], c->comm, as_stream(stream)));
    return MPX_OK;
}

// non-blocking health check: MPX_OK, or the communicator's asynchronous error
extern "C" int mpx_comm_check(void *h) {
    MPX_CHECK_ARG(h, "null communicator");
    ncclResult_t ar = ncclSuccess;
    MPX_NCCL(g_api.CommGetAsyncError(static_cast<Comm *>(h)->comm, &ar));
    if (ar != ncclSuccess) {
        set_error("RCCL asynchronous error: %s", g_api.GetErrorString(ar));
        return MPX_ERR_HIP;
    }
    return MPX_OK;
}

// Failure recovery: abort a communicator whose peers stopped responding (a
// hung or dead rank). Outstanding RCCL kernels are released; the handle is
// freed. Safe to call from a watchdog thread while another thread is blocked
// on the stream.
extern "C" int mpx_comm_abort(void *h) {
    if (!h) return MPX_OK;
    Comm *c = static_cast<Comm *>(h);
    (void)hipSetDevice(c->device);
    if (c->comm) g_api.CommAbort(c->comm);
    c->comm = nullptr;
    return MPX_OK;
}

// The communicator's comm stream (highest priority, non-blocking): callers that
// software-pipeline exchanges across steps order work on it with their own
// events (e.g. torch.cuda.ExternalStream + Event).
extern "C" void *mpx_comm_stream(void *h) { return h ? static_cast<Comm *>(h)->cstream : nullptr; }
