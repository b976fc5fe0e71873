"""Multi-GPU sharding for the batch engine (one process per GPU).

Frames are independent: a batch is split into contiguous index
ranges, one per rank, with no exchange of frame data.  The only collective is the
final sum of the per-flow counters, u64[(n_buckets+1)*4]: on GPUs it is the C ABI's
rpkt_gpu_flow_reduce (one RCCL all-reduce over xGMI) on torch.distributed's own
RCCL communicator; a gloo group (CPU tests, one-GPU rehearsals) sums through
torch.distributed instead.

Which path a reduce takes is decided once for the whole group: every rank states
whether it can call the C ABI on an RCCL communicator, the group takes the minimum of
those flags, and all ranks then issue the same collective.  A rank-local refusal can
therefore never leave some ranks in ncclAllReduce and others in torch's all_reduce
(which would hang both).  The path taken, and why, is kept in `last_reduce_path` /
`last_reduce_error`.
"""
import torch
import torch.distributed as dist

last_reduce_path = None      # "rccl" | "torch" | "gloo" | "local" after reduce_counters
last_reduce_error = None     # why the group did not take the C ABI path (None if it did)


def shard_range(n, rank, world):
    """Contiguous [lo, hi) of n frames owned by `rank` (sizes differ by at most 1)."""
    return n * rank // world, n * (rank + 1) // world


def agree(ok, group=None):
    """True on every rank iff `ok` holds on every rank of the group (one tiny all-reduce
    of a flag, MIN, on the group's own backend)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return bool(ok)
    dev = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
    t = torch.tensor([1 if ok else 0], dtype=torch.int32, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
    return bool(int(t.item()))


def _c_abi_comm(group):
    """(comm, None) when this rank can hand the group's RCCL communicator to the C ABI,
    else (None, reason)."""
    try:
        from . import engine
        engine.lib()
        comm = engine.nccl_comm_of(group)
    except Exception as e:                       # no engine / no communicator API
        return None, "%s: %s" % (type(e).__name__, e)
    if comm is None:
        return None, "no RCCL communicator for this device"
    return comm, None


def reduce_counters(counters, group=None, *, n_buckets=None, stream=None, via="auto"):
    """Sum flow counters over all ranks in place (u64 stored as int64: two's complement
    addition is exact for the unsigned values) and return them.

    via="auto": on an nccl group, the C ABI's rpkt_gpu_flow_reduce on the group's RCCL
    communicator when every rank can make that call, else torch.distributed.all_reduce
    on every rank (the reason lands in last_reduce_error); via="torch" forces the torch
    all-reduce.  A gloo group (CPU rehearsals) always sums through torch.distributed.
    The path taken is in dist.last_reduce_path."""
    global last_reduce_path, last_reduce_error
    if isinstance(group, int) and not isinstance(group, bool):
        # the round-2 signature reduce_counters(counters, n_buckets): still accepted
        import warnings
        warnings.warn("reduce_counters(counters, n_buckets) is deprecated: pass "
                      "n_buckets=... (the second positional argument is the process group)",
                      DeprecationWarning, stacklevel=2)
        group, n_buckets = None, group
    last_reduce_error = None
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        last_reduce_path = "local"
        return counters
    if counters.is_cuda and dist.get_backend(group) == "nccl":
        comm, why = _c_abi_comm(group) if via == "auto" else (None, "torch path requested")
        if agree(comm is not None, group):
            from . import engine
            nb = counters.numel() // 4 - 1 if n_buckets is None else n_buckets
            # the group agreed to take this path: a failure here raises rather than
            # falling back, since the other ranks are already inside ncclAllReduce
            engine.flow_reduce(counters, nb, comm, stream=stream)
            last_reduce_path = "rccl"
            return counters
        last_reduce_error = why or "another rank cannot use the C ABI reduce"
        dist.all_reduce(counters, op=dist.ReduceOp.SUM, group=group)
        last_reduce_path = "torch"
        return counters
    if counters.is_cuda:                             # gloo sums host tensors
        host = counters.cpu()
        dist.all_reduce(host, op=dist.ReduceOp.SUM, group=group)
        counters.copy_(host)
    else:
        dist.all_reduce(counters, op=dist.ReduceOp.SUM, group=group)
    last_reduce_path = dist.get_backend(group)
    return counters


def counters_as_u64(counters):
    t = counters.detach().cpu().contiguous()
    return t.numpy().view("uint64").reshape(-1, 4)
