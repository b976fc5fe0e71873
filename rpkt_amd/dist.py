"""Multi-GPU sharding for the batch engine (one process per GPU).

Frames are independent: a batch is split into contiguous index
ranges, one per rank, with no exchange of frame data.  The only collective is the
final sum of the per-flow counters, u64[(n_buckets+1)*4]: on GPUs it is the C ABI's
rpkt_gpu_flow_reduce (one RCCL all-reduce over xGMI) on torch.distributed's own
RCCL communicator; a gloo group (CPU tests, one-GPU rehearsals) sums through
torch.distributed instead.

The communicator can also be the library's own (via="own"): rank 0 makes an RCCL id
with rpkt_gpu_coll_unique_id, the group broadcasts it, and every rank joins it with
rpkt_gpu_comm_init, so the reduce does not depend on torch's private communicator
accessor or on ProcessGroupNCCL's stream bookkeeping.

Which path a reduce takes is decided once for the whole group: every rank states
whether it can call the C ABI on an RCCL communicator, the group takes the minimum of
those flags, and all ranks then issue the same collective.  A rank-local refusal can
therefore never leave some ranks in ncclAllReduce and others in torch's all_reduce
(which would hang both).  The path taken, and why, is kept in `last_reduce_path` /
`last_reduce_error`.
"""
import torch
import torch.distributed as dist

last_reduce_path = None      # "rccl_own" | "rccl" | "torch" | "gloo" | "local" after reduce_counters
_own_comms = {}              # process group -> the library's own ncclComm_t (as int)
last_reduce_error = None     # why the group did not take the C ABI path (None if it did)
last_exchange_error = None   # on rank 0: why make_id() failed in the last exchange_id
# how long rpkt_gpu_comm_init_timeout waits for every rank to join before it aborts
COMM_INIT_TIMEOUT_MS = 60000


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


def exchange_id(make_id, group=None, nbytes=128):
    """Rank 0 of the group calls make_id() (the RCCL unique id, `nbytes` bytes) and the
    group broadcasts it: every rank returns the same bytes, or None on every rank when
    rank 0 could not make one (a flag travels with the id, so no rank waits alone).  Rank
    0 keeps the reason in `last_exchange_error`."""
    global last_exchange_error
    last_exchange_error = None
    dev = "cuda" if dist.get_backend(group) == "nccl" else "cpu"
    buf = torch.zeros(1 + nbytes, dtype=torch.uint8)
    if dist.get_rank(group) == 0:
        try:
            uid = bytes(make_id())
            if len(uid) != nbytes:
                raise ValueError("id of %d bytes, want %d" % (len(uid), nbytes))
            buf[0] = 1
            buf[1:] = torch.tensor(list(uid), dtype=torch.uint8)
        except Exception as e:                   # the flag stays 0: every rank gets None
            last_exchange_error = "%s: %s" % (type(e).__name__, e)
    buf = buf.to(dev)
    src = dist.get_global_rank(group, 0) if group is not None else 0
    dist.broadcast(buf, src=src, group=group)
    buf = buf.cpu()
    return bytes(buf[1:].tolist()) if int(buf[0]) else None


def own_comm(group=None, timeout_ms=None, _engine=None):
    """(comm, None): the library's own RCCL communicator over the group's ranks (made on
    first use, then cached), or (None, reason) on every rank when the group cannot make
    one.  Every rank must first be able to call RCCL through the engine (agreed), then
    rank 0's id is broadcast and all ranks join it with rpkt_gpu_comm_init_timeout: a
    rank whose peer never joins (it failed before its init) gets its half-made
    communicator aborted after `timeout_ms` instead of blocking, and the group then
    agrees whether every rank holds a communicator, so either all ranks use it or none
    does (a rank that made one aborts it).  `_engine` replaces the engine module in CPU
    tests."""
    key = group if group is not None else dist.group.WORLD
    if key in _own_comms:
        return _own_comms[key], None
    engine = _engine
    try:
        if engine is None:
            from . import engine
        can = engine.lib().rpkt_gpu_coll_version() > 0
        why = None if can else "RCCL not loadable by the engine"
    except Exception as e:                       # no engine on this rank
        can, why, engine = False, "%s: %s" % (type(e).__name__, e), None
    if not agree(can, group):
        return None, why or "another rank cannot load RCCL"
    uid = exchange_id(engine.coll_unique_id, group, engine.COLL_ID_BYTES)
    if uid is None:
        return None, "rank 0 could not make an RCCL unique id%s" % (
            ": " + last_exchange_error if last_exchange_error else "")
    comm, why = None, None
    try:
        comm = engine.comm_init_timeout(dist.get_world_size(group), uid, dist.get_rank(group),
                                        COMM_INIT_TIMEOUT_MS if timeout_ms is None else timeout_ms)
    except Exception as e:                       # timed out, or the init failed
        why = "comm init on rank %d: %s: %s" % (dist.get_rank(group), type(e).__name__, e)
    if not agree(comm is not None, group):
        if comm is not None:                     # the group gives it up: no collective on it
            try:
                engine.comm_abort(comm)
            except Exception:
                pass
        return None, why or "another rank's rpkt_gpu_comm_init_timeout failed"
    _own_comms[key] = comm
    return comm, None


def release_own_comms():
    """rpkt_gpu_comm_destroy for every communicator own_comm made."""
    from . import engine
    for comm in _own_comms.values():
        engine.comm_destroy(comm)
    _own_comms.clear()


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
    on every rank (the reason lands in last_reduce_error); via="own": the same call on
    the library's own communicator (own_comm), falling back to "auto" when the group
    cannot make one; via="torch" forces the torch all-reduce.  A gloo group (CPU
    rehearsals) always sums through torch.distributed.  The path taken is in
    dist.last_reduce_path ("rccl_own", "rccl", "torch", "gloo", "local")."""
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
        own_why = None
        if via == "own":
            comm, own_why = own_comm(group)
            if comm is not None:
                from . import engine
                nb = counters.numel() // 4 - 1 if n_buckets is None else n_buckets
                engine.flow_reduce(counters, nb, comm, stream=stream)
                last_reduce_path = "rccl_own"
                return counters
        comm, why = _c_abi_comm(group) if via in ("auto", "own") else (None, "torch path requested")
        if own_why:
            why = "own communicator: %s; %s" % (own_why, why or "torch's communicator taken")
        if agree(comm is not None, group):
            from . import engine
            nb = counters.numel() // 4 - 1 if n_buckets is None else n_buckets
            # the group agreed to take this path: a failure here raises rather than
            # falling back, since the other ranks are already inside ncclAllReduce
            engine.flow_reduce(counters, nb, comm, stream=stream)
            last_reduce_path = "rccl"
            if own_why:
                last_reduce_error = why
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
