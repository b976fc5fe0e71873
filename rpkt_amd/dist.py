"""Multi-GPU sharding for the batch engine (one process per GPU).

Frames are independent: a batch is split into contiguous index
ranges, one per rank, with no exchange of frame data.  The only collective is the
final sum of the per-flow counters, u64[(n_buckets+1)*4]: on GPUs it is the C ABI's
rpkt_gpu_flow_reduce (one RCCL all-reduce over xGMI) on torch.distributed's own
RCCL communicator; a gloo group (CPU tests, one-GPU rehearsals) sums through
torch.distributed instead.
"""
import torch.distributed as dist


def shard_range(n, rank, world):
    """Contiguous [lo, hi) of n frames owned by `rank` (sizes differ by at most 1)."""
    return n * rank // world, n * (rank + 1) // world


def reduce_counters(counters, n_buckets=None, group=None, stream=None):
    """Sum flow counters over all ranks in place (u64 stored as int64: two's
    complement addition is exact for the unsigned values).  Returns the path taken:
    "rccl" (rpkt_gpu_flow_reduce on the group's RCCL communicator), "gloo"
    (torch.distributed.all_reduce) or "local" (one rank)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return "local"
    if counters.is_cuda and dist.get_backend(group) == "nccl":
        from . import engine
        nb = counters.numel() // 4 - 1 if n_buckets is None else n_buckets
        comm = engine.nccl_comm_of(group)
        if comm is None:
            raise engine.RpktError("RCCL process group has no communicator for this device")
        engine.flow_reduce(counters, nb, comm, stream=stream)
        return "rccl"
    if counters.is_cuda:                             # gloo sums host tensors
        host = counters.cpu()
        dist.all_reduce(host, op=dist.ReduceOp.SUM, group=group)
        counters.copy_(host)
    else:
        dist.all_reduce(counters, op=dist.ReduceOp.SUM, group=group)
    return dist.get_backend(group)


def counters_as_u64(counters):
    t = counters.detach().cpu().contiguous()
    return t.numpy().view("uint64").reshape(-1, 4)
