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

#include <dlfcn.h>
#include <mutex>
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
        R.ok = R.get_version && R.comm_count && R.all_reduce && R.reduce && R.get_unique_id &&
               R.comm_init_rank && R.comm_destroy;
    });
    return R;
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
    if (r != ncclSuccess) {
        g_last_coll_error = (int)r;
        return RPKT_E_COLL;
    }
    return RPKT_OK;
}

}  // extern "C"
