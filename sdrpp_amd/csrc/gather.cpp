// Spectra gather over RCCL (xGMI), the only collective of the multi-GPU layout:
// one rank per GPU / IQ stream; rank 0 (the display) receives every rank's rows. SDR++ itself
// has no multi-device code, so this is the C-ABI a C++ host (one process per GPU, or one thread
// per GPU in one process) calls instead of going through torch.distributed.
//
// RCCL is opened at first use (dlopen), not linked: the library loads on hosts without RCCL, and
// a process that already holds an RCCL (PyTorch's bundled librccl) shares it instead of loading
// a second copy. SDRGPU_RCCL_LIB names another build to load instead (tests load a stub with a
// peer that never answers). The communicator is built from a 128-byte id that rank 0 creates
// (sdrgpu_gather_get_id) and the host distributes out of band (any channel: a socket, MPI,
// torch.distributed's store), like ncclCommInitRank.
//
// A gather is one ncclGroupStart/End of point-to-point sends to rank 0 and the matching receives
// there (rank 0's own rows are a device copy), on the caller's stream: asynchronous, ordered
// after the producer of the rows on that stream.
//
// Failure model. The reference's blocks stop by flagging their streams and joining their worker
// threads (utils/threading.h:53-62, dsp/stream.h:94-116): nothing waits forever on a peer that is
// gone. Here the peers are other processes, so every wait on them has a deadline
// (SDRGPU_GATHER_TIMEOUT_S, default 120 s, or sdrgpu_gather_set_timeout): the communicator is
// non-blocking (ncclConfig_t.blocking = 0), init and group end are polled with
// ncclCommGetAsyncError, and sdrgpu_gather_wait polls the stream the same way. On expiry the
// communicator is aborted (ncclCommAbort) and the call returns SDRGPU_ETIMEOUT naming the rank,
// instead of blocking the process; later calls on the handle fail with SDRGPU_ESTATE.
#include <dlfcn.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <rccl/rccl.h>
#include "sdrgpu_internal.h"

using namespace sdrgpu;

namespace {
struct Rccl {
    void* lib = nullptr;
    decltype(&ncclGetUniqueId) getUniqueId = nullptr;
    decltype(&ncclCommInitRank) commInitRank = nullptr;
    decltype(&ncclCommInitRankConfig) commInitRankConfig = nullptr;   // (non-blocking init; optional)
    decltype(&ncclCommGetAsyncError) getAsyncError = nullptr;
    decltype(&ncclCommAbort) commAbort = nullptr;
    decltype(&ncclCommDestroy) commDestroy = nullptr;
    decltype(&ncclSend) send = nullptr;
    decltype(&ncclRecv) recv = nullptr;
    decltype(&ncclGroupStart) groupStart = nullptr;
    decltype(&ncclGroupEnd) groupEnd = nullptr;
    decltype(&ncclGetErrorString) errorString = nullptr;
};

const Rccl* rccl() {
    static Rccl r;
    static std::once_flag once;
    static char why[256] = "missing symbols";
    std::call_once(once, [] {
        if (const char* p = std::getenv("SDRGPU_RCCL_LIB")) {   // another build (tests: a stub)
            r.lib = dlopen(p, RTLD_NOW | RTLD_LOCAL);
        } else {
            // an RCCL already in the process first (RTLD_NOLOAD), then the ROCm one
            const char* names[] = {"librccl.so", "librccl.so.1"};
            for (const char* n : names)
                if (!r.lib) r.lib = dlopen(n, RTLD_NOW | RTLD_NOLOAD | RTLD_GLOBAL);
            for (const char* n : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
                if (!r.lib) r.lib = dlopen(n, RTLD_NOW | RTLD_GLOBAL);
        }
        if (!r.lib) {
            // dlerror() clears the error state on every call: read it once
            const char* e = dlerror();
            std::snprintf(why, sizeof(why), "%s", e ? e : "dlopen failed");
            return;
        }
        auto sym = [](const char* n) { return dlsym(r.lib, n); };
        r.getUniqueId = (decltype(r.getUniqueId))sym("ncclGetUniqueId");
        r.commInitRank = (decltype(r.commInitRank))sym("ncclCommInitRank");
        r.commInitRankConfig = (decltype(r.commInitRankConfig))sym("ncclCommInitRankConfig");
        r.getAsyncError = (decltype(r.getAsyncError))sym("ncclCommGetAsyncError");
        r.commAbort = (decltype(r.commAbort))sym("ncclCommAbort");
        r.commDestroy = (decltype(r.commDestroy))sym("ncclCommDestroy");
        r.send = (decltype(r.send))sym("ncclSend");
        r.recv = (decltype(r.recv))sym("ncclRecv");
        r.groupStart = (decltype(r.groupStart))sym("ncclGroupStart");
        r.groupEnd = (decltype(r.groupEnd))sym("ncclGroupEnd");
        r.errorString = (decltype(r.errorString))sym("ncclGetErrorString");
    });
    if (!r.lib || !r.getUniqueId || !r.commInitRank || !r.getAsyncError || !r.commAbort || !r.commDestroy || !r.send ||
        !r.recv || !r.groupStart || !r.groupEnd || !r.errorString) {
        set_error("gather: RCCL (librccl.so) not available: %s", why);
        return nullptr;
    }
    return &r;
}

double env_timeout() {
    if (const char* e = std::getenv("SDRGPU_GATHER_TIMEOUT_S")) {
        const double t = std::atof(e);
        if (t > 0) return t;
    }
    return 120.0;
}

using Clock = std::chrono::steady_clock;
Clock::time_point deadline_after(double s) {
    return Clock::now() + std::chrono::duration_cast<Clock::duration>(std::chrono::duration<double>(s));
}

// back-off of the polls: the first ones yield (a group end normally completes in microseconds,
// and the host thread issuing the next step's launches must not sleep behind it), later ones sleep
void poll_pause(int k) {
    if (k < 256) std::this_thread::yield();
    else std::this_thread::sleep_for(std::chrono::microseconds(100));
}

// polls the communicator's state until it leaves ncclInProgress or the deadline passes
ncclResult_t wait_comm(const Rccl* R, ncclComm_t c, Clock::time_point dl, bool* expired) {
    *expired = false;
    for (int k = 0;; k++) {
        ncclResult_t st = ncclSuccess;
        const ncclResult_t e = R->getAsyncError(c, &st);
        if (e != ncclSuccess) return e;
        if (st != ncclInProgress) return st;
        if (Clock::now() >= dl) {
            *expired = true;
            return ncclInProgress;
        }
        poll_pause(k);
    }
}
}  // namespace

struct sdrgpu_gather {
    int device = 0, rank = 0, world = 1;
    ncclComm_t comm = nullptr;
    double timeout = 120.0;   // seconds, every wait on the peers
    bool aborted = false;     // the communicator was aborted: the handle only accepts destroy
};

static_assert(sizeof(ncclUniqueId) == SDRGPU_GATHER_ID_BYTES, "RCCL unique id size");

// the communicator is unusable (a peer timed out or failed): abort it (never blocks, unlike
// ncclCommDestroy, which waits for the operations a dead peer will not complete)
static int gather_fail(const Rccl* R, sdrgpu_gather* g, int rc, const char* what, ncclResult_t e, bool expired) {
    if (g->comm && !g->aborted) (void)R->commAbort(g->comm);
    g->aborted = true;
    if (expired)
        set_error("gather: rank %d of %d: %s did not complete within %.1f s (a peer rank is missing or stalled); "
                  "communicator aborted", g->rank, g->world, what, g->timeout);
    else
        set_error("gather: rank %d of %d: %s failed: %s; communicator aborted", g->rank, g->world, what, R->errorString(e));
    return rc;
}

extern "C" int sdrgpu_gather_get_id(void* id) {
    if (!id) { set_error("gather_get_id: null id"); return SDRGPU_EARG; }
    const Rccl* R = rccl();
    if (!R) return SDRGPU_ESTATE;
    ncclUniqueId u;
    const ncclResult_t e = R->getUniqueId(&u);
    if (e != ncclSuccess) { set_error("ncclGetUniqueId failed: %s", R->errorString(e)); return SDRGPU_EHIP; }
    std::memcpy(id, &u, sizeof(u));
    return SDRGPU_OK;
}

// device < 0: the calling thread's current HIP device (the host bound it already)
extern "C" int sdrgpu_gather_create(sdrgpu_gather** out, int device, int rank, int world, const void* id) {
    if (!out || !id || world < 1 || rank < 0 || rank >= world) { set_error("gather_create: bad argument"); return SDRGPU_EARG; }
    *out = nullptr;
    const Rccl* R = rccl();
    if (!R) return SDRGPU_ESTATE;
    if (device >= 0) SDRGPU_SET_DEVICE(device);
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    auto* g = new sdrgpu_gather();
    g->device = device; g->rank = rank; g->world = world;
    g->timeout = env_timeout();
    const auto dl = deadline_after(g->timeout);
    ncclResult_t e;
    bool expired = false;
    // non-blocking: the init's rendezvous with the peers is polled (SDRGPU_GATHER_BLOCKING=1: the
    // blocking init, no deadline before the communicator exists)
    const char* blk = std::getenv("SDRGPU_GATHER_BLOCKING");
    if (R->commInitRankConfig && !(blk && std::atoi(blk) != 0)) {
        ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
        cfg.blocking = 0;
        e = R->commInitRankConfig(&g->comm, world, u, rank, &cfg);
        if ((e == ncclSuccess || e == ncclInProgress) && g->comm) e = wait_comm(R, g->comm, dl, &expired);
    } else {
        e = R->commInitRank(&g->comm, world, u, rank);
    }
    if (e != ncclSuccess) {
        const int rc = gather_fail(R, g, expired ? SDRGPU_ETIMEOUT : SDRGPU_EHIP, "ncclCommInitRank", e, expired);
        delete g;
        return rc;
    }
    *out = g;
    return SDRGPU_OK;
}

extern "C" int sdrgpu_gather_set_timeout(sdrgpu_gather* g, double seconds) {
    if (!g || !(seconds > 0)) { set_error("gather_set_timeout: bad argument"); return SDRGPU_EARG; }
    g->timeout = seconds;
    return SDRGPU_OK;
}

extern "C" int sdrgpu_gather_rows(sdrgpu_gather* g, const float* rows, long long count, float* out, void* stream) {
    if (!g || (count > 0 && !rows) || count < 0 || (g->rank == 0 && count > 0 && !out)) {
        set_error("gather_rows: bad argument");
        return SDRGPU_EARG;
    }
    if (g->aborted) { set_error("gather_rows: rank %d: communicator aborted after an earlier failure", g->rank); return SDRGPU_ESTATE; }
    if (count == 0) return SDRGPU_OK;
    const Rccl* R = rccl();
    if (!R) return SDRGPU_ESTATE;
    if (g->device >= 0) SDRGPU_SET_DEVICE(g->device);
    hipStream_t s = (hipStream_t)stream;
    ncclResult_t e = R->groupStart();
    if (e != ncclSuccess) return gather_fail(R, g, SDRGPU_EHIP, "ncclGroupStart", e, false);
    // A non-blocking communicator may answer ncclInProgress for a send/recv: that is an operation
    // accepted into the group, so every peer's operation is still posted after it; only a real error
    // stops the posting (and aborts the communicator).
    ncclResult_t bad = ncclSuccess;
    auto post = [&](ncclResult_t r) {
        if (r != ncclSuccess && r != ncclInProgress && bad == ncclSuccess) bad = r;
    };
    if (g->world == 1) {   // one stream: a send/recv to itself (exercises the communicator like world > 1)
        post(R->send(rows, (size_t)count, ncclFloat32, 0, g->comm, s));
        if (bad == ncclSuccess) post(R->recv(out, (size_t)count, ncclFloat32, 0, g->comm, s));
    } else if (g->rank == 0) {
        for (int r = 1; bad == ncclSuccess && r < g->world; r++)
            post(R->recv(out + (size_t)r * count, (size_t)count, ncclFloat32, r, g->comm, s));
    } else {
        post(R->send(rows, (size_t)count, ncclFloat32, 0, g->comm, s));
    }
    if (bad != ncclSuccess) {
        (void)R->groupEnd();
        return gather_fail(R, g, SDRGPU_EHIP, "ncclSend/ncclRecv", bad, false);
    }
    e = R->groupEnd();
    bool expired = false;
    if (e == ncclInProgress) e = wait_comm(R, g->comm, deadline_after(g->timeout), &expired);
    if (e != ncclSuccess) return gather_fail(R, g, expired ? SDRGPU_ETIMEOUT : SDRGPU_EHIP, "ncclGroupEnd", e, expired);
    // rank 0's own rows: a device copy on the same stream (independent of the received slots)
    if (g->rank == 0 && g->world > 1) SDRGPU_HIP(hipMemcpyAsync(out, rows, sizeof(float) * count, hipMemcpyDeviceToDevice, s));
    return SDRGPU_OK;
}

// Waits for the gathers enqueued on `stream` (and anything before them there) with the handle's
// deadline: the stream and the communicator's asynchronous error are polled, so a peer that died
// after its group was enqueued ends the wait with SDRGPU_ETIMEOUT (communicator aborted) instead of
// a stream that never drains. timeoutS <= 0: the handle's timeout.
extern "C" int sdrgpu_gather_wait(sdrgpu_gather* g, void* stream, double timeoutS) {
    if (!g) { set_error("gather_wait: null handle"); return SDRGPU_EARG; }
    if (g->aborted) { set_error("gather_wait: rank %d: communicator aborted after an earlier failure", g->rank); return SDRGPU_ESTATE; }
    const Rccl* R = rccl();
    if (!R) return SDRGPU_ESTATE;
    if (g->device >= 0) SDRGPU_SET_DEVICE(g->device);
    const double t = timeoutS > 0 ? timeoutS : g->timeout;
    const auto dl = deadline_after(t);
    for (int k = 0;; k++) {
        const hipError_t q = hipStreamQuery((hipStream_t)stream);
        if (q == hipSuccess) return SDRGPU_OK;
        if (q != hipErrorNotReady) {
            set_error("gather_wait: hipStreamQuery failed: %s", hipGetErrorName(q));
            return SDRGPU_EHIP;
        }
        ncclResult_t st = ncclSuccess;
        const ncclResult_t e = R->getAsyncError(g->comm, &st);
        if (e != ncclSuccess || (st != ncclSuccess && st != ncclInProgress))
            return gather_fail(R, g, SDRGPU_EHIP, "the enqueued gather", e != ncclSuccess ? e : st, false);
        if (Clock::now() >= dl) {
            const double keep = g->timeout;
            g->timeout = t;
            const int rc = gather_fail(R, g, SDRGPU_ETIMEOUT, "the enqueued gather", ncclInProgress, true);
            g->timeout = keep;
            return rc;
        }
        poll_pause(k);
    }
}

extern "C" int sdrgpu_gather_destroy(sdrgpu_gather* g) {
    if (!g) return SDRGPU_OK;
    if (g->comm && !g->aborted) {
        if (const Rccl* R = rccl()) R->commDestroy(g->comm);
    }
    delete g;
    return SDRGPU_OK;
}
