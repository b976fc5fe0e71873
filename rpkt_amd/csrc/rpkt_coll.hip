// rpkt_coll.hip — the path's one collective: the per-flow counter sum over ranks.
//
// Frames never cross GPUs: each rank parses its own shard and
// accumulates u64[(n_buckets + 1) * 4] counters with rpkt_gpu_flow_count.  The
// only exchange is this sum, one RCCL all-reduce (or reduce to a root) of the
// counter array on the caller's communicator and stream, over xGMI.  It replaces
// the per-queue counters a DPDK receive loop keeps per thread and adds up at the
// end (rpkt-dpdk/examples/loopback_tx.rs:176-181, rss_rx.rs:54-113).
//
// The library links librccl.so.1 by soname: under PyTorch the communicator comes
// from ProcessGroupNCCL and the soname resolves to the RCCL torch already loaded;
// a C/C++/Rust host gets /opt/rocm's RCCL and its own ncclCommInit*.
#include "rpkt_common.h"

#include <rccl/rccl.h>

namespace {
thread_local int g_last_coll_error = 0;
}  // namespace

extern "C" {

int rpkt_gpu_last_coll_error(void) { return g_last_coll_error; }

int rpkt_gpu_coll_version(void) {
    int v = 0;
    return ncclGetVersion(&v) == ncclSuccess ? v : -1;
}

int rpkt_gpu_flow_reduce(uint64_t* counters_dev, uint32_t n_buckets, int root, void* nccl_comm,
                         void* stream) {
    if (!counters_dev || !nccl_comm || n_buckets == 0 || n_buckets > RPKT_FLOW_MAX_BUCKETS ||
        root < -1)
        return RPKT_E_INVAL;
    if (((uintptr_t)counters_dev & 7u) != 0) return RPKT_E_ALIGN;
    ncclComm_t comm = (ncclComm_t)nccl_comm;
    int nranks = 0;
    ncclResult_t r = ncclCommCount(comm, &nranks);
    if (r == ncclSuccess && root >= nranks) return RPKT_E_INVAL;
    const size_t count = ((size_t)n_buckets + 1) * 4;
    hipStream_t s = (hipStream_t)stream;
    if (r == ncclSuccess)
        r = root < 0 ? ncclAllReduce(counters_dev, counters_dev, count, ncclUint64, ncclSum, comm, s)
                     : ncclReduce(counters_dev, counters_dev, count, ncclUint64, ncclSum, root,
                                  comm, s);
    if (r != ncclSuccess) {
        g_last_coll_error = (int)r;
        return RPKT_E_COLL;
    }
    return RPKT_OK;
}

}  // extern "C"
