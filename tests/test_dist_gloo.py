"""world_size-2 gloo run of the multi-GPU logic on CPU: each rank generates only
its shard of the IMIX batch (config 4), computes flow events + counters for it
(the oracle stands in for the GPU here), and the counters are all-reduced; the
result must equal the single-process counters of the whole batch."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

N = 60000
NB = 8192


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle
    from rpkt_amd import dist as rd, gen
    lo, hi = rd.shard_range(N, rank, world)
    hb = gen.make_batch(4, hi - lo, first=lo)
    _, ev = oracle.parse_batch(hb.frames, hb.n, flags=3, offsets=hb.offsets, n_buckets=NB,
                               flow_ev=True)
    c = torch.from_numpy(oracle.flow_count(ev, NB).view(np.int64).copy())
    assert rd.reduce_counters(c) is c and rd.last_reduce_path == "gloo"
    # the round-2 call form reduce_counters(counters, n_buckets) still works, with a warning
    import warnings
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        ones = torch.ones((NB + 1) * 4, dtype=torch.int64)
        assert rd.reduce_counters(ones, NB) is ones and (ones == world).all()
        assert any(issubclass(x.category, DeprecationWarning) for x in w)
    if rank == 0:
        np.save(out, c.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_counters_equal_whole_batch(tmp_path, world):
    from oracle import oracle
    from rpkt_amd import gen
    out = str(tmp_path / "c.npy")
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    got = np.load(out).view(np.uint64)
    hb = gen.make_batch(4, N)
    _, ev = oracle.parse_batch(hb.frames, hb.n, flags=3, offsets=hb.offsets, n_buckets=NB,
                               flow_ev=True)
    assert np.array_equal(got, oracle.flow_count(ev, NB))


def test_shard_ranges_partition():
    from rpkt_amd.dist import shard_range
    for n in (0, 1, 7, 1000, 8 << 20):
        for w in (1, 2, 3, 8):
            r = [shard_range(n, k, w) for k in range(w)]
            assert r[0][0] == 0 and r[-1][1] == n
            assert all(r[k][1] == r[k + 1][0] for k in range(w - 1))
            assert max(b - a for a, b in r) - min(b - a for a, b in r) <= 1


def _agree_worker(rank, world, port, flags, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rpkt_amd import dist as rd
    got = rd.agree(flags[rank])
    with open("%s.%d" % (out, rank), "w") as fh:
        fh.write("1" if got else "0")
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("flags", [(True, True), (True, False), (False, True), (True, True, False)])
def test_reduce_path_is_decided_for_the_whole_group(tmp_path, flags):
    """dist.agree (the C-ABI-reduce decision): every rank gets the same answer, True only
    when every rank can take the RCCL path, so a rank-local refusal never splits the
    ranks between ncclAllReduce and torch's all_reduce."""
    out = str(tmp_path / "agree")
    world = len(flags)
    mp.spawn(_agree_worker, args=(world, _free_port(), flags, out), nprocs=world, join=True)
    got = {open("%s.%d" % (out, r)).read() for r in range(world)}
    assert got == {"1" if all(flags) else "0"}


def _id_worker(rank, world, port, fail, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rpkt_amd import dist as rd

    def make_id():                       # stands in for rpkt_gpu_coll_unique_id (rank 0 only)
        assert rank == 0
        if fail:
            raise RuntimeError("no RCCL")
        return bytes(range(128))
    got = rd.exchange_id(make_id)
    with open("%s.%d" % (out, rank), "wb") as fh:
        fh.write(b"NONE" if got is None else got)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,fail", [(2, False), (3, False), (2, True)])
def test_own_communicator_id_exchange(tmp_path, world, fail):
    """The library-owned communicator's id (dist.exchange_id): rank 0 makes it, every rank
    receives the same 128 bytes; when rank 0 cannot make one every rank gets None (no rank
    goes on to rpkt_gpu_comm_init alone)."""
    out = str(tmp_path / "id")
    mp.spawn(_id_worker, args=(world, _free_port(), fail, out), nprocs=world, join=True)
    got = {open("%s.%d" % (out, r), "rb").read() for r in range(world)}
    assert got == {b"NONE" if fail else bytes(range(128))}


class _StubLib:
    def rpkt_gpu_coll_version(self):
        return 22700


class _StubEngine:
    """Stands in for rpkt_amd.engine in own_comm: rank `fail_rank`'s comm init fails (as a
    peer that never joins makes the others' rpkt_gpu_comm_init_timeout time out), or rank
    0's id cannot be made."""
    COLL_ID_BYTES = 128

    def __init__(self, rank, fail_rank, fail_id, log):
        self.rank, self.fail_rank, self.fail_id, self.log = rank, fail_rank, fail_id, log

    def lib(self):
        return _StubLib()

    def coll_unique_id(self):
        if self.fail_id:
            raise RuntimeError("rpkt_gpu_coll_unique_id failed: RCCL error (ncclResult 2)")
        return bytes(range(128))

    def comm_init_timeout(self, world, uid, rank, timeout_ms):
        assert uid == bytes(range(128)) and timeout_ms > 0
        if rank == self.fail_rank:
            raise RuntimeError("rpkt_gpu_comm_init_timeout failed: RCCL error (ncclResult 7)")
        return 0x1000 + rank

    def comm_abort(self, comm):
        self.log.append(("abort", comm))


def _own_worker(rank, world, port, fail_rank, fail_id, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from rpkt_amd import dist as rd
    log = []
    comm, why = rd.own_comm(timeout_ms=5000,
                            _engine=_StubEngine(rank, fail_rank, fail_id, log))
    with open("%s.%d" % (out, rank), "w") as fh:
        fh.write("%s|%s|%s" % (comm, why, ",".join("%s:%s" % x for x in log)))
    rd._own_comms.clear()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,fail_rank,fail_id", [(2, -1, False), (2, 1, False),
                                                     (3, 0, False), (3, 2, False),
                                                     (2, -1, True)])
def test_own_comm_init_failure_is_agreed(tmp_path, world, fail_rank, fail_id):
    """One rank's communicator init fails (or rank 0 cannot make the id): own_comm returns
    (None, reason) on EVERY rank, the ranks whose init succeeded abort their half of the
    communicator, and rank 0's reason names the cause; with no failure every rank keeps
    its communicator."""
    out = str(tmp_path / "own")
    mp.spawn(_own_worker, args=(world, _free_port(), fail_rank, fail_id, out), nprocs=world,
             join=True)
    res = [open("%s.%d" % (out, r)).read().split("|") for r in range(world)]
    if fail_rank < 0 and not fail_id:
        assert [c for c, _, _ in res] == [str(0x1000 + r) for r in range(world)]
        assert all(w == "None" and a == "" for _, w, a in res)
        return
    assert all(c == "None" for c, _, _ in res)
    for r, (_, why, aborted) in enumerate(res):
        assert why != "None"
        if fail_id:
            assert aborted == ""
            if r == 0:
                assert "ncclResult 2" in why
        elif r == fail_rank:
            assert "ncclResult 7" in why and aborted == ""
        else:
            assert aborted == "abort:%d" % (0x1000 + r)
