// dp.hip -- the data-parallel gradient exchange issued natively over RCCL (include/gsr.h,
// "native exchange").  gsr_tools/dp.py's ShExchange / all-reduce paths issue the same
// collectives through torch.distributed, whose Python call path costs 25-35 us of host time per
// collective and ~60 us for the SH completion's stream bookkeeping: at one view per rank and
// step the host then becomes the bottleneck (RCCL world-1 rehearsal: the SH exchange's start
// took 130-170 us of a 0.9-ms step, profiles/round4_c_rccl_world1_sh.json).  Here one C call
// orders a communication stream after the caller's, issues the collectives as one RCCL group and
// the dsh rebuild behind them, and records a ticket event the caller's stream waits on later.
//
// librccl is loaded on first use (dlopen), so libgsr has no link-time dependency on it and a
// process that never calls gsr_dp_init never loads it.  The communicator is the library's own
// (ncclCommInitRank with a unique id the caller broadcasts, e.g. over torch.distributed), beside
// whatever process group the caller uses for everything else.
#include "gsr_internal.h"
#include "../../include/gsr_train.h"

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <cstring>
#include <mutex>
#include <string>

namespace gsr {
namespace {

struct Rccl {
    void* lib = nullptr;
    ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) =
        nullptr;
    ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    const char* (*ErrorString)(ncclResult_t) = nullptr;
};

// Tickets: a ring of events; a ticket stays valid until DP_TICKETS later exchanges.
constexpr int DP_TICKETS = 16;

struct DpState {
    std::mutex mu;
    Rccl r;
    ncclComm_t comm = nullptr;
    int world = 0, rank = 0, device = -1;
    hipStream_t cs = nullptr;  // communication stream
    hipEvent_t ready = nullptr;
    hipEvent_t done[DP_TICKETS] = {};
    int next = 0;
};
DpState& dp() {
    static DpState s;
    return s;
}

int dp_fail(const std::string& m) { return set_error("[gsr] dp: " + m); }

int load_rccl(Rccl& r) {
    if (r.lib) return 0;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
    if (!h) return dp_fail(std::string("cannot load librccl: ") + dlerror());
    auto sym = [&](const char* n) { return dlsym(h, n); };
    r.GetUniqueId = reinterpret_cast<decltype(r.GetUniqueId)>(sym("ncclGetUniqueId"));
    r.CommInitRank = reinterpret_cast<decltype(r.CommInitRank)>(sym("ncclCommInitRank"));
    r.CommDestroy = reinterpret_cast<decltype(r.CommDestroy)>(sym("ncclCommDestroy"));
    r.AllReduce = reinterpret_cast<decltype(r.AllReduce)>(sym("ncclAllReduce"));
    r.AllGather = reinterpret_cast<decltype(r.AllGather)>(sym("ncclAllGather"));
    r.GroupStart = reinterpret_cast<decltype(r.GroupStart)>(sym("ncclGroupStart"));
    r.GroupEnd = reinterpret_cast<decltype(r.GroupEnd)>(sym("ncclGroupEnd"));
    r.ErrorString = reinterpret_cast<decltype(r.ErrorString)>(sym("ncclGetErrorString"));
    if (!r.GetUniqueId || !r.CommInitRank || !r.CommDestroy || !r.AllReduce || !r.AllGather || !r.GroupStart ||
        !r.GroupEnd || !r.ErrorString) {
        dlclose(h);
        return dp_fail("librccl lacks an expected symbol");
    }
    r.lib = h;
    return 0;
}

int nccl_check(const Rccl& r, ncclResult_t e, const char* what) {
    if (e == ncclSuccess) return 0;
    return dp_fail(std::string(what) + ": " + (r.ErrorString ? r.ErrorString(e) : "error"));
}

// Destroy the communicator, the stream and the events (whichever exist); the state is then
// uninitialised.  Caller holds s.mu.
ncclResult_t release(DpState& s) {
    ncclResult_t e = ncclSuccess;
    if (s.comm) e = s.r.CommDestroy(s.comm);
    s.comm = nullptr;
    for (int i = 0; i < DP_TICKETS; ++i)
        if (s.done[i]) (void)hipEventDestroy(s.done[i]), s.done[i] = nullptr;
    if (s.ready) (void)hipEventDestroy(s.ready), s.ready = nullptr;
    if (s.cs) (void)hipStreamDestroy(s.cs), s.cs = nullptr;
    s.world = 0;
    return e;
}

// Order the communication stream after `stream`'s work so far.
int dp_begin(DpState& s, hipStream_t stream) {
    if (!s.comm) return dp_fail("not initialised (gsr_dp_init)");
    int dev = -1;
    if (hipGetDevice(&dev) != hipSuccess || dev != s.device) return dp_fail("called on another device than gsr_dp_init's");
    if (hipEventRecord(s.ready, stream) != hipSuccess || hipStreamWaitEvent(s.cs, s.ready, 0) != hipSuccess)
        return dp_fail("stream ordering failed");
    return 0;
}

// Record the ticket event after the communication stream's work; returns the ticket or -1.
int dp_end(DpState& s) {
    const int t = s.next;
    s.next = (s.next + 1) % DP_TICKETS;
    if (hipEventRecord(s.done[t], s.cs) != hipSuccess) {
        dp_fail("ticket event record failed");
        return -1;
    }
    return t;
}

}  // namespace
}  // namespace gsr

extern "C" {

size_t gsr_dp_unique_id_bytes(void) { return sizeof(ncclUniqueId); }

int gsr_dp_get_unique_id(void* out) {
    using namespace gsr;
    (void)set_error("");
    if (!out) return dp_fail("null unique-id buffer");
    DpState& s = dp();
    std::lock_guard<std::mutex> lk(s.mu);
    if (int rc = load_rccl(s.r)) return rc;
    ncclUniqueId id;
    if (int rc = nccl_check(s.r, s.r.GetUniqueId(&id), "ncclGetUniqueId")) return rc;
    std::memcpy(out, &id, sizeof(id));
    return 0;
}

int gsr_dp_init(const void* unique_id, int world, int rank) {
    using namespace gsr;
    (void)set_error("");
    if (!unique_id || world < 1 || rank < 0 || rank >= world) return dp_fail("bad unique id / world / rank");
    DpState& s = dp();
    std::lock_guard<std::mutex> lk(s.mu);
    if (s.comm) return dp_fail("already initialised (gsr_dp_finalize first)");
    if (int rc = load_rccl(s.r)) return rc;
    if (hipGetDevice(&s.device) != hipSuccess) return dp_fail("no current device");
    ncclUniqueId id;
    std::memcpy(&id, unique_id, sizeof(id));
    if (int rc = nccl_check(s.r, s.r.CommInitRank(&s.comm, world, id, rank), "ncclCommInitRank")) {
        s.comm = nullptr;
        return rc;
    }
    bool ok = hipStreamCreateWithFlags(&s.cs, hipStreamNonBlocking) == hipSuccess &&
              hipEventCreateWithFlags(&s.ready, hipEventDisableTiming) == hipSuccess;
    for (int i = 0; ok && i < DP_TICKETS; ++i) ok = hipEventCreateWithFlags(&s.done[i], hipEventDisableTiming) == hipSuccess;
    if (!ok) {
        // leave nothing half-initialised: a retry starts from scratch
        release(s);
        return dp_fail("stream / event creation failed");
    }
    s.world = world;
    s.rank = rank;
    s.next = 0;
    return 0;
}

int gsr_dp_world(void) {
    gsr::DpState& s = gsr::dp();
    std::lock_guard<std::mutex> lk(s.mu);
    return s.comm ? s.world : 0;
}

int gsr_dp_finalize(void) {
    using namespace gsr;
    (void)set_error("");
    DpState& s = dp();
    std::lock_guard<std::mutex> lk(s.mu);
    if (!s.comm) return 0;
    if (s.cs) (void)hipStreamSynchronize(s.cs);
    return nccl_check(s.r, release(s), "ncclCommDestroy");
}

int gsr_dp_allreduce(float* buf, size_t n, void* stream) {
    using namespace gsr;
    (void)set_error("");
    DpState& s = dp();
    std::lock_guard<std::mutex> lk(s.mu);
    if (n > 0 && !buf) {
        dp_fail("null buffer");
        return -1;
    }
    if (dp_begin(s, (hipStream_t)stream)) return -1;
    if (n > 0 && nccl_check(s.r, s.r.AllReduce(buf, buf, n, ncclFloat32, ncclSum, s.comm, s.cs), "ncclAllReduce"))
        return -1;
    return dp_end(s);
}

int gsr_dp_sh_exchange(int P, int D, int M, int C, const float* means3D, int views_per_rank, float* arena,
                       const float* rows, float* rows_all, void* stream) {
    using namespace gsr;
    (void)set_error("");
    DpState& s = dp();
    std::lock_guard<std::mutex> lk(s.mu);
    if (P < 0 || D < 0 || D > 3 || M < 1 || M < (D + 1) * (D + 1) || C < 0 || views_per_rank < 1) {
        dp_fail("bad P / D / M / C / views");
        return -1;
    }
    if (P > 0 && (!means3D || !arena || !rows || !rows_all)) {
        dp_fail("null argument");
        return -1;
    }
    if (dp_begin(s, (hipStream_t)stream)) return -1;
    if (P > 0) {
        long long off[GSR_ARENA_BLOCKS + 1];
        gsr_arena_layout(P, M, C, off);
        // [dmeans3D] and [dopacity .. bucket end) are summed; dsh is rebuilt from the rows
        const size_t n_rows = (size_t)views_per_rank * sh_rows_floats(P);
        const Rccl& r = s.r;
        if (nccl_check(r, r.GroupStart(), "ncclGroupStart")) return -1;
        ncclResult_t e = r.AllReduce(arena + off[0], arena + off[0], 3 * (size_t)P, ncclFloat32, ncclSum, s.comm, s.cs);
        if (e == ncclSuccess)
            e = r.AllReduce(arena + off[2], arena + off[2], (size_t)(off[GSR_ARENA_BLOCKS] - off[2]), ncclFloat32,
                            ncclSum, s.comm, s.cs);
        if (e == ncclSuccess) e = r.AllGather(rows, rows_all, n_rows, ncclFloat32, s.comm, s.cs);
        const ncclResult_t ge = r.GroupEnd();
        if (nccl_check(r, e, "SH exchange collectives") || nccl_check(r, ge, "ncclGroupEnd")) return -1;
        launch_sh_backward(P, D, M, means3D, s.world * views_per_rank, rows_all, arena + off[1], s.cs);
        const hipError_t he = hipGetLastError();
        if (he != hipSuccess) {
            dp_fail(std::string("dsh rebuild: ") + hipGetErrorString(he));
            return -1;
        }
    }
    return dp_end(s);
}

int gsr_dp_wait(int ticket, void* stream) {
    using namespace gsr;
    (void)set_error("");
    DpState& s = dp();
    std::lock_guard<std::mutex> lk(s.mu);
    if (!s.comm) return dp_fail("not initialised (gsr_dp_init)");
    if (ticket < 0 || ticket >= DP_TICKETS || !s.done[ticket]) return dp_fail("bad ticket");
    if (hipStreamWaitEvent((hipStream_t)stream, s.done[ticket], 0) != hipSuccess) return dp_fail("stream wait failed");
    return 0;
}

}  // extern "C"
