"""Multi-rank paths on the GPU: ranks that each run the real HIP parse + flow-count on
their shard and sum counters across ranks, the bench's own N-rank launcher, and the
C ABI's RCCL reduce on torch.distributed's communicator.  The lease has one GPU, so
the 2-rank cases share cuda:0 over gloo (RCCL refuses two ranks on one device); the
RCCL call itself runs on a world-1 communicator here and on 8 GPUs in the driver's
scaling run."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N = 300000
NB = 8192


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    from rpkt_amd import dist as rd, engine, gen
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = rd.shard_range(N, rank, world)
    hb = gen.make_batch(4, hi - lo, first=lo)
    db = engine.DeviceBatch.from_host(hb)
    _, ev = engine.parse_batch(db, 3 | 4, n_buckets=NB)
    c = engine.flow_count(ev, hb.n, NB)
    rd.reduce_counters(c, n_buckets=NB)
    via = rd.last_reduce_path
    torch.cuda.synchronize()
    if rank == 0:
        np.save(out, c.cpu().numpy())
        with open(out + ".via", "w") as fh:
            fh.write(via)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_ranks_hip_flow_counters_equal_whole_batch(tmp_path, world):
    """Each rank: its shard of the config-4 IMIX batch through rpkt_gpu_parse_batch
    (flow events) + rpkt_gpu_flow_count on cuda:0; counters summed over the ranks must
    equal the oracle's counters of the whole batch, word for word."""
    from oracle import oracle
    from rpkt_amd import gen
    out = str(tmp_path / "c.npy")
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    got = np.load(out).view(np.uint64)
    assert open(out + ".via").read() == "gloo"
    hb = gen.make_batch(4, N)
    _, ev = oracle.parse_batch(hb.frames, hb.n, flags=3, offsets=hb.offsets, n_buckets=NB,
                               flow_ev=True, threads=8)
    want = oracle.flow_count(ev, NB).reshape(-1, 4)
    assert int(want[:, 0].sum()) == N
    assert np.array_equal(got.reshape(-1, 4), want)


@pytest.mark.parametrize("world", [2, 3])
def test_bench_launches_n_ranks(tmp_path, world):
    """bench.py --gpus N starts its own N ranks (no torchrun) and runs the N-rank default
    leg set (the headline, config 4's shards + counter reduce, the strong legs): the
    counter sum covers every frame of every launch of every rank and is verified against
    torch's sum, and rank 0's one stdout line parses and fits the driver's 8,000-char
    tail."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    detail = str(tmp_path / "detail.json")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world),
                        "--dist-backend", "gloo", "--no-cpu", "--frames", "200000", "--steps",
                        "3", "--warmup", "1", "--min-warmup-s", "0", "--detail", detail],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    out = r.stdout.strip().splitlines()
    assert len(out) == 1 and len(out[0]) < 8000, out
    line = json.loads(out[0])
    assert line["n_gpus"] == world and line["config"]["dist_backend"] == "gloo"
    assert set(line["extra"]) == {"config4", "config2_strong", "config3_strong"}
    assert line["config"]["frames_per_rank"] == 200000 and "copy_ceiling_gb_per_s" not in line
    assert line["flow_pkts_total"] == line["flow_pkts_expected"] > 0
    assert line["flow_reduce_via"] == "gloo" and line["flow_reduce_verified"] is True
    assert line["roofline"]["frac"] > 0 and line["cpu_baseline"] is None
    with open(detail) as fh:
        full = json.load(fh)
    assert full["n_gpus"] == world and "roofline" in full["extra"]["config4"]


RCCL_SCRIPT = r"""
import os, sys
sys.path.insert(0, %r)
import numpy as np, torch, torch.distributed as dist
from rpkt_amd import engine
torch.cuda.set_device(0)
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=%r, RANK="0", WORLD_SIZE="1")
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
comm = engine.nccl_comm_of()
assert comm, "no RCCL communicator"
nb = 8192
rng = np.random.default_rng(5)
host = rng.integers(0, 2**62, (nb + 1) * 4, dtype=np.int64)
c = torch.from_numpy(host.copy()).cuda()
engine.flow_reduce(c, nb, comm)                    # all-reduce over the world-1 comm
engine.flow_reduce(c, nb, comm, root=0)            # reduce to rank 0
torch.cuda.synchronize()
assert np.array_equal(c.cpu().numpy(), host)
try:
    engine.flow_reduce(c, nb, comm, root=1)        # no rank 1 in this world
    raise SystemExit("root 1 accepted")
except engine.RpktError:
    pass
print("rccl ok", engine.lib().rpkt_gpu_coll_version())
dist.destroy_process_group()
"""


def test_flow_reduce_on_torch_rccl_communicator(tmp_path):
    """rpkt_gpu_flow_reduce on the ncclComm_t of torch.distributed's RCCL group (the
    communicator the bench's N-rank config 4 hands the C ABI)."""
    script = tmp_path / "rccl.py"
    script.write_text(RCCL_SCRIPT % (ROOT, str(_free_port())))
    r = subprocess.run([sys.executable, str(script)], capture_output=True, text=True,
                       timeout=180, cwd=ROOT)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    assert "rccl ok" in r.stdout


THREADS_SCRIPT = r"""
import sys, threading
sys.path.insert(0, %r)
import numpy as np, torch
from rpkt_amd import engine, gen
from oracle import oracle
torch.cuda.set_device(0)
NB = 8192
hbs = [gen.make_batch(4, 200000, seed=40 + t) for t in range(2)]
dbs = [engine.DeviceBatch.from_host(h) for h in hbs]
evs = [engine.parse_batch(d, 3 | 4, n_buckets=NB)[1] for d in dbs]
torch.cuda.synchronize()
go = threading.Barrier(2)
out = [None, None]
def run(t):
    s = torch.cuda.Stream()
    go.wait()                  # both threads make the process's first flow_count call at once
    c = engine.flow_count(evs[t], hbs[t].n, NB, stream=s)
    s.synchronize()
    out[t] = c.cpu().numpy().view(np.uint64)
th = [threading.Thread(target=run, args=(t,)) for t in range(2)]
[x.start() for x in th]
[x.join() for x in th]
for t in range(2):
    _, ev = oracle.parse_batch(hbs[t].frames, hbs[t].n, flags=3, offsets=hbs[t].offsets,
                               n_buckets=NB, flow_ev=True)
    assert np.array_equal(out[t], oracle.flow_count(ev, NB)), t
print("threads ok")
"""


def test_flow_count_from_two_host_threads(tmp_path):
    """Two host threads make the process's first rpkt_gpu_flow_count calls at the same time
    on their own streams (the per-device, locked one-time LDS attribute setup); both
    counter sets equal the oracle's."""
    script = tmp_path / "threads.py"
    script.write_text(THREADS_SCRIPT % ROOT)
    r = subprocess.run([sys.executable, str(script)], capture_output=True, text=True,
                       timeout=180, cwd=ROOT)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    assert "threads ok" in r.stdout


OWN_SCRIPT = r"""
import os, sys
sys.path.insert(0, %r)
import numpy as np, torch, torch.distributed as dist
from rpkt_amd import dist as rd, engine
torch.cuda.set_device(0)
# the library's own communicator through the C ABI alone (no torch group)
uid = engine.coll_unique_id()
assert len(uid) == engine.COLL_ID_BYTES and any(uid)
comm = engine.comm_init(1, uid, 0)
nb = 4096
rng = np.random.default_rng(6)
host = rng.integers(0, 2**62, (nb + 1) * 4, dtype=np.int64)
c = torch.from_numpy(host.copy()).cuda()
engine.flow_reduce(c, nb, comm)
torch.cuda.synchronize()
assert np.array_equal(c.cpu().numpy(), host)
engine.comm_destroy(comm)
# and as the dist path makes it: id from rank 0, broadcast over the torch group
os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=%r, RANK="0", WORLD_SIZE="1")
dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
comm2, why = rd.own_comm()
assert comm2 and why is None, why
engine.flow_reduce(c, nb, comm2, root=0)
torch.cuda.synchronize()
assert np.array_equal(c.cpu().numpy(), host)
rd.release_own_comms()
dist.destroy_process_group()
# the deadline join: world 1 joins at once (non-blocking communicator, polled) and its
# all-reduce keeps the blocking contract; a world-2 id whose peer never comes is aborted
# after the deadline and reports ncclInProgress (7), not a hang
comm3 = engine.comm_init_timeout(1, engine.coll_unique_id(), 0, 20000)
engine.flow_reduce(c, nb, comm3)
torch.cuda.synchronize()
assert np.array_equal(c.cpu().numpy(), host)
engine.comm_destroy(comm3)
import time
t0 = time.time()
try:
    engine.comm_init_timeout(2, engine.coll_unique_id(), 0, 2000)
    raise SystemExit("a world-2 init with no peer returned a communicator")
except engine.RpktError as e:
    assert engine.last_coll_error() == 7, (str(e), engine.last_coll_error())
assert time.time() - t0 < 60, time.time() - t0
print("own comm ok")
"""


def test_flow_reduce_on_the_library_own_communicator(tmp_path):
    """rpkt_gpu_coll_unique_id + rpkt_gpu_comm_init (world 1) + rpkt_gpu_flow_reduce +
    rpkt_gpu_comm_destroy, directly and through dist.own_comm over an RCCL group."""
    script = tmp_path / "own.py"
    script.write_text(OWN_SCRIPT % (ROOT, str(_free_port())))
    r = subprocess.run([sys.executable, str(script)], capture_output=True, text=True,
                       timeout=180, cwd=ROOT)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    assert "own comm ok" in r.stdout


def _probe(world, **env):
    e = dict(os.environ, **{k: str(v) for k, v in env.items()})
    e.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "rccl_share_probe.py"),
                        str(world)], capture_output=True, text=True, timeout=240, env=e, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert sorted(x["rank"] for x in lines) == list(range(world)), lines
    return lines


@pytest.mark.parametrize("world", [2, 3])
def test_rccl_ranks_sharing_one_gpu(world):
    """N RCCL ranks on the one leased GPU (a distinct NCCL_HOSTID per rank: RCCL sees N
    hosts and talks over loopback sockets): each rank's shard of config 4 parsed and counted
    by the HIP engine, the counters summed by rpkt_gpu_flow_reduce over ncclAllReduce on
    torch's communicator (auto) and on the library's own, joined across the ranks with
    rpkt_gpu_comm_init_timeout (own); both equal torch's all_reduce and cover every frame."""
    for x in _probe(world):
        assert x["auto"]["path"] == "rccl" and x["own"]["path"] == "rccl_own", x
        for via in ("auto", "own"):
            assert x[via]["pkts"] == 400000 and x[via]["equal_torch"] is True, x


def test_own_comm_peer_never_joins_real_rccl():
    """Rank 1 fails before joining the library's communicator: rank 0's RCCL join is
    aborted at its 3-s deadline, the group agrees, and every rank falls back to torch's
    communicator (path rccl) with the right sums -- no hang."""
    lines = _probe(2, RPKT_PROBE_FAIL_RANK=1, RPKT_PROBE_TIMEOUT_MS=3000)
    for x in lines:
        assert x["own"]["path"] == "rccl" and x["own"]["pkts"] == 400000, x
        assert x["own"]["equal_torch"] is True and "own communicator" in x["own"]["error"], x
        assert x["own"]["seconds"] < 60, x
    assert "ncclResult 7" in [x for x in lines if x["rank"] == 0][0]["own"]["error"]


@pytest.mark.parametrize("comm", ["auto", "own"])
def test_bench_nccl_ranks_sharing_one_gpu(tmp_path, comm):
    """bench.py --gpus 2 --share-gpu: the N-rank default job over RCCL (nccl backend) on
    the one GPU, both counter-reduce paths: the line parses, every counter word equals
    torch's sum, and the frame total covers every launch of every rank."""
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--share-gpu", "--reduce-comm", comm, "--no-cpu", "--frames", "200000",
                        "--steps", "3", "--warmup", "1", "--min-warmup-s", "0", "--detail",
                        str(tmp_path / "d.json")], capture_output=True, text=True, timeout=300,
                       env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    out = r.stdout.strip().splitlines()
    assert len(out) == 1, out[:8]                  # RCCL's banner goes to stderr
    line = json.loads(out[0])
    assert line["n_gpus"] == 2 and line["config"]["dist_backend"] == "nccl"
    assert line["config"]["shared_gpu"] is True
    assert line["flow_reduce_via"] == ("rccl_own" if comm == "own" else "rccl"), line
    assert line["flow_reduce_verified"] is True
    assert line["flow_pkts_total"] == line["flow_pkts_expected"] > 0
    # the reduce as the median of 20 timed reduces (min <= median <= max), and the summed
    # achieved GB/s of both ranks beside the per-rank fraction
    assert line["flow_reduce_samples"] == 20
    assert 0 < line["flow_reduce_ms_min"] <= line["flow_reduce_ms"] <= line["flow_reduce_ms_max"]
    rf = line["roofline"]
    assert rf["peak_all_ranks"] == 2 * rf["peak"] and rf["achieved_all_ranks"] > rf["achieved"]
    assert len(json.dumps(line)) < 8000


def test_bench_under_torchrun_as_the_driver_launches_it(tmp_path):
    """The driver's own N>1 launch form: python -m torch.distributed.run --nnodes=1
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port P bench.py --gpus 2 ... --
    here with --share-gpu (both ranks on the one GPU, RCCL over loopback).  bench.py must
    take RANK / LOCAL_RANK / WORLD_SIZE from torchrun (not start ranks of its own) and print
    exactly one stdout line, rank 0's, with the counters verified."""
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node", "2", "--master-addr", "127.0.0.1", "--master-port",
                        str(port), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--share-gpu",
                        "--no-cpu", "--frames", "200000", "--steps", "3", "--warmup", "1",
                        "--min-warmup-s", "0", "--detail", str(tmp_path / "d.json")],
                       capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    out = r.stdout.strip().splitlines()
    assert len(out) == 1, out[:8]
    line = json.loads(out[0])
    assert line["n_gpus"] == 2 and line["config"]["dist_backend"] == "nccl"
    assert line["flow_reduce_via"] == "rccl" and line["flow_reduce_verified"] is True, line
    assert line["flow_pkts_total"] == line["flow_pkts_expected"] > 0
    assert len(json.dumps(line)) < 8000
