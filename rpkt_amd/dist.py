"""Multi-GPU sharding for the batch engine (one process per GPU).

Frames are independent: a batch is split into contiguous index
ranges, one per rank, with no exchange of frame data.  The only collective is the
final sum of the per-flow counters, an all-reduce of u64[(n_buckets+1)*4] over
RCCL (torch.distributed backend "nccl") on xGMI, or gloo on CPU for tests.
"""
import torch
import torch.distributed as dist


def shard_range(n, rank, world):
    """Contiguous [lo, hi) of n frames owned by `rank` (sizes differ by at most 1)."""
    return n * rank // world, n * (rank + 1) // world


def reduce_counters(counters, group=None):
    """Sum flow counters over all ranks in place (u64 stored as int64: two's
    complement addition is exact for the unsigned values)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(counters, op=dist.ReduceOp.SUM, group=group)
    return counters


def counters_as_u64(counters):
    t = counters.detach().cpu().contiguous()
    return t.numpy().view("uint64").reshape(-1, 4)
