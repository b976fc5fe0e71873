// rpkt_coll.hip — the path's one collective: the per-flow counter sum over ranks.
//
// Frames never cross GPUs: each rank parses its own shard and
// accumulates u64[(n_buckets + 1) * 4] counters with rpkt_gpu_flow_count.  The
// only exchange is this sum, one RCCL all-reduce (or reduce to a root) of the
// counter array on the caller's communicator and stream, over xGMI.  It replaces
// the per-queue counters a DPDK receive loop keeps per thread and adds up at the
// end (rpkt-dpdk/examples/loopback_tx.rs:176-181, rss_rx.rs:54-113).
//
// RCCL is resolved when the collective is first used, not at load time, so a parse-only
// host (C, C++, Rust) loads the engine without RCCL installed.  The communicator must
// belong to the RCCL copy in the process: one already loaded (PyTorch's, whose
// ProcessGroupNCCL made the communicator; found with RTLD_NOLOAD) is preferred over
// loading librccl.so.1 afresh (/opt/rocm's, for hosts that call ncclCommInit*
// themselves).  Without RCCL the calls return RPKT_E_COLL.
#include "rpkt_common.h"

#include <chrono>
#include <dlfcn.h>
#include <mutex>
#include <thread>
#include <rccl/rccl.h>        // types and enums only: every function goes through Rccl

namespace {
thread_local int g_last_coll_error = 0;

struct Rccl {
    decltype(&ncclGetVersion) get_version = nullptr;
    decltype(&ncclCommCount) comm_count = nullptr;
    decltype(&ncclAllReduce) all_reduce = nullptr;
    decltype(&ncclReduce) reduce = nullptr;
    decltype(&ncclGetUniqueId) get_unique_id = nullptr;
    decltype(&ncclCommInitRank) comm_init_rank = nullptr;
    decltype(&ncclCommDestroy) comm_destroy = nullptr;
    // non-blocking init with a deadline (rpkt_gpu_comm_init_timeout); optional
    decltype(&ncclCommInitRankConfig) comm_init_config = nullptr;
    decltype(&ncclCommGetAsyncError) async_error = nullptr;
    decltype(&ncclCommAbort) comm_abort = nullptr;
    bool ok = false;
};
static_assert(sizeof(ncclUniqueId) == RPKT_COLL_ID_BYTES, "RCCL unique id size");

const Rccl& rccl() {
    static Rccl R;
    static std::once_flag once;
    std::call_once(once, [] {
        void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_NOLOAD);
        if (!h) h = dlopen("librccl.so.1", RTLD_NOW | RTLD_LOCAL);
        if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_LOCAL);
        if (!h) return;
        R.get_version = (decltype(R.get_version))dlsym(h, "ncclGetVersion");
        R.comm_count = (decltype(R.comm_count))dlsym(h, "ncclCommCount");
        R.all_reduce = (decltype(R.all_reduce))dlsym(h, "ncclAllReduce");
        R.reduce = (decltype(R.reduce))dlsym(h, "ncclReduce");
        R.get_unique_id = (decltype(R.get_unique_id))dlsym(h, "ncclGetUniqueId");
        R.comm_init_rank = (decltype(R.comm_init_rank))dlsym(h, "ncclCommInitRank");
        R.comm_destroy = (decltype(R.comm_destroy))dlsym(h, "ncclCommDestroy");
        R.comm_init_config = (decltype(R.comm_init_config))dlsym(h, "ncclCommInitRankConfig");
        R.async_error = (decltype(R.async_error))dlsym(h, "ncclCommGetAsyncError");
        R.comm_abort = (decltype(R.comm_abort))dlsym(h, "ncclCommAbort");
        R.ok = R.get_version && R.comm_count && R.all_reduce && R.reduce && R.get_unique_id &&
               R.comm_init_rank && R.comm_destroy;
    });
    return R;
}

// Wait while a non-blocking communicator reports ncclInProgress (its init, or a call
// enqueued on it), at most `timeout_ms` (< 0: no limit).  Blocking communicators (torch's)
// never return ncclInProgress, so this is a no-op for them.
ncclResult_t settle(const Rccl& R, ncclComm_t comm, ncclResult_t r, int timeout_ms) {
    if (r != ncclInProgress || !R.async_error) return r;
    const auto t_end = std::chrono::steady_clock::now() + std::chrono::milliseconds(timeout_ms);
    for (;;) {
        ncclResult_t a = ncclInProgress;
        if (R.async_error(comm, &a) != ncclSuccess) return ncclSystemError;
        if (a != ncclInProgress) return a;
        if (timeout_ms >= 0 && std::chrono::steady_clock::now() >= t_end) return ncclInProgress;
        std::this_thread::sleep_for(std::chrono::microseconds(200));
    }
}
}  // namespace

extern "C" {

int rpkt_gpu_last_coll_error(void) { return g_last_coll_error; }

int rpkt_gpu_coll_version(void) {
    const Rccl& R = rccl();
    int v = 0;
    return R.ok && R.get_version(&v) == ncclSuccess ? v : -1;
}

// ---- a communicator the library owns (the caller does not need one from elsewhere) ----
int rpkt_gpu_coll_unique_id(uint8_t* id_out) {
    if (!id_out) return RPKT_E_INVAL;
    const Rccl& R = rccl();
    if (!R.ok) {
        g_last_coll_error = (int)ncclSystemError;
        return RPKT_E_COLL;
    }
    ncclUniqueId id;
    const ncclResult_t r = R.get_unique_id(&id);
    if (r != ncclSuccess) {
        g_last_coll_error = (int)r;
        return RPKT_E_COLL;
    }
    memcpy(id_out, &id, sizeof(id));
    return RPKT_OK;
}

int rpkt_gpu_comm_init(void** comm_out, int world, const uint8_t* id, int rank) {
    if (!comm_out || !id || world < 1 || rank < 0 || rank >= world) return RPKT_E_INVAL;
    *comm_out = nullptr;
    const Rccl& R = rccl();
    if (!R.ok) {
        g_last_coll_error = (int)ncclSystemError;
        return RPKT_E_COLL;
    }
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof(uid));
    ncclComm_t comm = nullptr;
    const ncclResult_t r = R.comm_init_rank(&comm, world, uid, rank);
    if (r != ncclSuccess) {
        g_last_coll_error = (int)r;
        return RPKT_E_COLL;
    }
    *comm_out = comm;
    return RPKT_OK;
}

// The same join with a deadline: the communicator is made non-blocking (config.blocking
// = 0) and its bootstrap polled; when a peer never arrives (it failed before joining),
// or the init fails, the half-made communicator is aborted and RPKT_E_COLL returned with
// rpkt_gpu_last_coll_error() = ncclInProgress (timed out) or the init's error, so every
// rank comes back and the group can agree on a fallback instead of hanging.
int rpkt_gpu_comm_init_timeout(void** comm_out, int world, const uint8_t* id, int rank,
                               int timeout_ms) {
    if (timeout_ms <= 0) return rpkt_gpu_comm_init(comm_out, world, id, rank);
    if (!comm_out || !id || world < 1 || rank < 0 || rank >= world) return RPKT_E_INVAL;
    *comm_out = nullptr;
    const Rccl& R = rccl();
    if (!R.ok || !R.comm_init_config || !R.async_error || !R.comm_abort) {
        g_last_coll_error = (int)ncclSystemError;
        return RPKT_E_COLL;
    }
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof(uid));
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    ncclComm_t comm = nullptr;
    ncclResult_t r = R.comm_init_config(&comm, world, uid, rank, &cfg);
    if (comm && (r == ncclSuccess || r == ncclInProgress)) r = settle(R, comm, ncclInProgress, timeout_ms);
    if (r != ncclSuccess) {
        g_last_coll_error = (int)r;
        if (comm) R.comm_abort(comm);
        return RPKT_E_COLL;
    }
    *comm_out = comm;
    return RPKT_OK;
}

// Tear a communicator down without waiting for its peers (after the group agreed to
// give it up, or when a peer is gone).
int rpkt_gpu_comm_abort(void* comm) {
    if (!comm) return RPKT_E_INVAL;
    const Rccl& R = rccl();
    if (!R.ok || !R.comm_abort) return RPKT_E_COLL;
    const ncclResult_t r = R.comm_abort((ncclComm_t)comm);
    if (r != ncclSuccess) {
        g_last_coll_error = (int)r;
        return RPKT_E_COLL;
    }
    return RPKT_OK;
}

int rpkt_gpu_comm_destroy(void* comm) {
    if (!comm) return RPKT_E_INVAL;
    const Rccl& R = rccl();
    if (!R.ok) return RPKT_E_COLL;
    const ncclResult_t r = R.comm_destroy((ncclComm_t)comm);
    if (r != ncclSuccess) {
        g_last_coll_error = (int)r;
        return RPKT_E_COLL;
    }
    return RPKT_OK;
}

int rpkt_gpu_flow_reduce(uint64_t* counters_dev, uint32_t n_buckets, int root, void* nccl_comm,
                         void* stream) {
    if (!counters_dev || !nccl_comm || n_buckets == 0 || n_buckets > RPKT_FLOW_MAX_BUCKETS ||
        root < -1)
        return RPKT_E_INVAL;
    if (((uintptr_t)counters_dev & 7u) != 0) return RPKT_E_ALIGN;
    const Rccl& R = rccl();
    if (!R.ok) {
        g_last_coll_error = (int)ncclSystemError;           // no RCCL in this process
        return RPKT_E_COLL;
    }
    ncclComm_t comm = (ncclComm_t)nccl_comm;
    int nranks = 0;
    ncclResult_t r = R.comm_count(comm, &nranks);
    if (r == ncclSuccess && root >= nranks) return RPKT_E_INVAL;
    const size_t count = ((size_t)n_buckets + 1) * 4;
    hipStream_t s = (hipStream_t)stream;
    if (r == ncclSuccess)
        r = root < 0 ? R.all_reduce(counters_dev, counters_dev, count, ncclUint64, ncclSum, comm, s)
                     : R.reduce(counters_dev, counters_dev, count, ncclUint64, ncclSum, root,
                                comm, s);
    // a non-blocking communicator (rpkt_gpu_comm_init_timeout) may return while the
    // enqueue is still in progress: wait for it here, so the call keeps the blocking
    // contract (queued on `stream` when it returns)
    r = settle(R, comm, r, -1);
    if (r != ncclSuccess) {
        g_last_coll_error = (int)r;
        return RPKT_E_COLL;
    }
    return RPKT_OK;
}

}  // extern "C"
