/* A stand-in RCCL for tests/test_gather_deadline.py (CPU suite): the C-ABI gather loads it through
 * SDRGPU_RCCL_LIB. Its "peer" never answers: in mode "init" (STUB_RCCL_MODE) the non-blocking
 * communicator never leaves ncclInProgress; in mode "group" init completes but every group end
 * stays in progress; in mode "post" init and group end complete but every send/recv answers
 * ncclInProgress (a non-blocking communicator accepting the operation). Each call is appended to the file STUB_RCCL_LOG so the test can check that
 * the library aborted the communicator. Only the symbols libsdrgpu resolves are defined, with the
 * ABI of rccl.h (enums as int, opaque handles as pointers). */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

typedef int res_t;          /* ncclResult_t */
enum { OK = 0, INVALID_USAGE = 5, IN_PROGRESS = 7 };
typedef struct { char internal[128]; } uid_t128;   /* ncclUniqueId */
static int comm_obj, aborted, in_group;

static void note(const char* what) {
    const char* p = getenv("STUB_RCCL_LOG");
    if (!p) return;
    FILE* f = fopen(p, "a");
    if (!f) return;
    fprintf(f, "%s\n", what);
    fclose(f);
}
static int mode_is(const char* m) {
    const char* e = getenv("STUB_RCCL_MODE");
    return e && strcmp(e, m) == 0;
}

res_t ncclGetUniqueId(uid_t128* u) { memset(u, 0x5a, sizeof(*u)); note("getUniqueId"); return OK; }
res_t ncclCommInitRank(void** comm, int n, uid_t128 id, int rank) {
    (void)n; (void)id; (void)rank;
    *comm = &comm_obj;
    note("initRank");
    return OK;
}
res_t ncclCommInitRankConfig(void** comm, int n, uid_t128 id, int rank, void* cfg) {
    (void)n; (void)id; (void)rank; (void)cfg;
    *comm = &comm_obj;
    note("initRankConfig");
    return mode_is("init") ? IN_PROGRESS : OK;
}
res_t ncclCommGetAsyncError(void* comm, res_t* st) {
    (void)comm;
    if (aborted) *st = INVALID_USAGE;
    else if (mode_is("init") || (mode_is("group") && in_group)) *st = IN_PROGRESS;
    else *st = OK;
    return OK;
}
res_t ncclCommAbort(void* comm) { (void)comm; aborted = 1; note("abort"); return OK; }
res_t ncclCommDestroy(void* comm) { (void)comm; note("destroy"); return OK; }
res_t ncclSend(const void* b, size_t n, int t, int peer, void* comm, void* s) {
    (void)b; (void)n; (void)t; (void)peer; (void)comm; (void)s; note("send"); return mode_is("post") ? IN_PROGRESS : OK;
}
res_t ncclRecv(void* b, size_t n, int t, int peer, void* comm, void* s) {
    (void)b; (void)n; (void)t; (void)peer; (void)comm; (void)s;
    char w[32];
    snprintf(w, sizeof(w), "recv%d", peer);
    note(w);
    return mode_is("post") ? IN_PROGRESS : OK;
}
res_t ncclGroupStart(void) { note("groupStart"); return OK; }
res_t ncclGroupEnd(void) {
    note("groupEnd");
    if (mode_is("group")) { in_group = 1; return IN_PROGRESS; }
    return OK;
}
const char* ncclGetErrorString(res_t r) { return r == IN_PROGRESS ? "in progress" : r == OK ? "success" : "error"; }
