// Spectra gather over RCCL (xGMI), the only collective of the multi-GPU layout:
// one rank per GPU / IQ stream; rank 0 (the display) receives every rank's rows. SDR++ itself
// has no multi-device code, so this is the C-ABI a C++ host (one process per GPU, or one thread
// per GPU in one process) calls instead of going through torch.distributed.
//
// RCCL is opened at first use (dlopen), not linked: the library loads on hosts without RCCL, and
// a process that already holds an RCCL (PyTorch's bundled librccl) shares it instead of loading
// a second copy. The communicator is built from a 128-byte id that rank 0 creates
// (sdrgpu_gather_get_id) and the host distributes out of band (any channel: a socket, MPI,
// torch.distributed's store), like ncclCommInitRank.
//
// A gather is one ncclGroupStart/End of point-to-point sends to rank 0 and the matching receives
// there (rank 0's own rows are a device copy), on the caller's stream: asynchronous, ordered
// after the producer of the rows on that stream.
#include <dlfcn.h>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <rccl/rccl.h>
#include "sdrgpu_internal.h"

using namespace sdrgpu;

namespace {
struct Rccl {
    void* lib = nullptr;
    decltype(&ncclGetUniqueId) getUniqueId = nullptr;
    decltype(&ncclCommInitRank) commInitRank = nullptr;
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
        // an RCCL already in the process first (RTLD_NOLOAD), then the ROCm one
        const char* names[] = {"librccl.so", "librccl.so.1"};
        for (const char* n : names)
            if (!r.lib) r.lib = dlopen(n, RTLD_NOW | RTLD_NOLOAD | RTLD_GLOBAL);
        for (const char* n : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"})
            if (!r.lib) r.lib = dlopen(n, RTLD_NOW | RTLD_GLOBAL);
        if (!r.lib) {
            // dlerror() clears the error state on every call: read it once
            const char* e = dlerror();
            std::snprintf(why, sizeof(why), "%s", e ? e : "dlopen failed");
            return;
        }
        r.getUniqueId = (decltype(r.getUniqueId))dlsym(r.lib, "ncclGetUniqueId");
        r.commInitRank = (decltype(r.commInitRank))dlsym(r.lib, "ncclCommInitRank");
        r.commDestroy = (decltype(r.commDestroy))dlsym(r.lib, "ncclCommDestroy");
        r.send = (decltype(r.send))dlsym(r.lib, "ncclSend");
        r.recv = (decltype(r.recv))dlsym(r.lib, "ncclRecv");
        r.groupStart = (decltype(r.groupStart))dlsym(r.lib, "ncclGroupStart");
        r.groupEnd = (decltype(r.groupEnd))dlsym(r.lib, "ncclGroupEnd");
        r.errorString = (decltype(r.errorString))dlsym(r.lib, "ncclGetErrorString");
    });
    if (!r.lib || !r.getUniqueId || !r.commInitRank || !r.commDestroy || !r.send || !r.recv || !r.groupStart ||
        !r.groupEnd || !r.errorString) {
        set_error("gather: RCCL (librccl.so) not available: %s", why);
        return nullptr;
    }
    return &r;
}

#define RCCL_CALL(R, call)                                                                   \
    do {                                                                                     \
        ncclResult_t e_ = (call);                                                            \
        if (e_ != ncclSuccess) {                                                             \
            set_error("%s failed: %s", #call, (R)->errorString(e_));                       \
            return SDRGPU_EHIP;                                                              \
        }                                                                                    \
    } while (0)
// closes an RCCL group on every exit path (an error inside the group must not leave the thread's
// group open for later RCCL calls)
struct GroupGuard {
    const Rccl* R;
    bool open = false;
    explicit GroupGuard(const Rccl* r) : R(r) {}
    ncclResult_t start() {
        const ncclResult_t e = R->groupStart();
        open = e == ncclSuccess;
        return e;
    }
    ncclResult_t end() {
        open = false;
        return R->groupEnd();
    }
    ~GroupGuard() {
        if (open) (void)R->groupEnd();
    }
};
}  // namespace

struct sdrgpu_gather {
    int device = 0, rank = 0, world = 1;
    ncclComm_t comm = nullptr;
};

static_assert(sizeof(ncclUniqueId) == SDRGPU_GATHER_ID_BYTES, "RCCL unique id size");

extern "C" int sdrgpu_gather_get_id(void* id) {
    if (!id) { set_error("gather_get_id: null id"); return SDRGPU_EARG; }
    const Rccl* R = rccl();
    if (!R) return SDRGPU_ESTATE;
    ncclUniqueId u;
    RCCL_CALL(R, R->getUniqueId(&u));
    std::memcpy(id, &u, sizeof(u));
    return SDRGPU_OK;
}

extern "C" int sdrgpu_gather_create(sdrgpu_gather** out, int device, int rank, int world, const void* id) {
    if (!out || !id || world < 1 || rank < 0 || rank >= world) { set_error("gather_create: bad argument"); return SDRGPU_EARG; }
    *out = nullptr;
    const Rccl* R = rccl();
    if (!R) return SDRGPU_ESTATE;
    SDRGPU_SET_DEVICE(device);
    ncclUniqueId u;
    std::memcpy(&u, id, sizeof(u));
    auto* g = new sdrgpu_gather();
    g->device = device; g->rank = rank; g->world = world;
    const ncclResult_t e = R->commInitRank(&g->comm, world, u, rank);
    if (e != ncclSuccess) {
        set_error("ncclCommInitRank(%d of %d) failed: %s", rank, world, R->errorString(e));
        delete g;
        return SDRGPU_EHIP;
    }
    *out = g;
    return SDRGPU_OK;
}

extern "C" int sdrgpu_gather_rows(sdrgpu_gather* g, const float* rows, long long count, float* out, void* stream) {
    if (!g || (count > 0 && !rows) || count < 0 || (g->rank == 0 && count > 0 && !out)) {
        set_error("gather_rows: bad argument");
        return SDRGPU_EARG;
    }
    if (count == 0) return SDRGPU_OK;
    const Rccl* R = rccl();
    if (!R) return SDRGPU_ESTATE;
    SDRGPU_SET_DEVICE(g->device);
    hipStream_t s = (hipStream_t)stream;
    GroupGuard grp(R);
    if (g->world == 1) {   // one stream: a send/recv to itself (exercises the communicator like world > 1)
        RCCL_CALL(R, grp.start());
        RCCL_CALL(R, R->send(rows, (size_t)count, ncclFloat32, 0, g->comm, s));
        RCCL_CALL(R, R->recv(out, (size_t)count, ncclFloat32, 0, g->comm, s));
        RCCL_CALL(R, grp.end());
        return SDRGPU_OK;
    }
    if (g->rank == 0) SDRGPU_HIP(hipMemcpyAsync(out, rows, sizeof(float) * count, hipMemcpyDeviceToDevice, s));
    RCCL_CALL(R, grp.start());
    if (g->rank == 0) {
        for (int r = 1; r < g->world; r++)
            RCCL_CALL(R, R->recv(out + (size_t)r * count, (size_t)count, ncclFloat32, r, g->comm, s));
    } else {
        RCCL_CALL(R, R->send(rows, (size_t)count, ncclFloat32, 0, g->comm, s));
    }
    RCCL_CALL(R, grp.end());
    return SDRGPU_OK;
}

extern "C" int sdrgpu_gather_destroy(sdrgpu_gather* g) {
    if (!g) return SDRGPU_OK;
    if (g->comm) {
        if (const Rccl* R = rccl()) R->commDestroy(g->comm);
    }
    delete g;
    return SDRGPU_OK;
}
