"""Probe (GPU box): two RCCL ranks on ONE GPU.  RCCL refuses two ranks of one host on one
device ("Duplicate GPU detected"); with a distinct NCCL_HOSTID per rank the ranks look
like two hosts and talk over the socket transport on loopback, so the cross-rank RCCL
path (ncclCommInitRank, ncclAllReduce through the C ABI, torch's ProcessGroupNCCL) runs
on a one-GPU box.  Not xGMI: a correctness rehearsal of the multi-rank code, not a
bandwidth measurement.

Usage: python tools/rccl_share_probe.py [world]   (prints one JSON line per rank)
  RPKT_PROBE_FAIL_RANK=r: rank r fails before it joins the library's own communicator
  (its rpkt_gpu_comm_init_timeout is never called), RPKT_PROBE_TIMEOUT_MS the others'
  join deadline: they must abort, agree and fall back together instead of hanging.
"""
import json
import os
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def share_env(rank, world, port):
    """Environment of rank `rank` of a `world`-rank job sharing one GPU over RCCL."""
    return dict(os.environ, RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                NCCL_HOSTID="rpkt-share-%d" % rank, NCCL_SOCKET_IFNAME="lo",
                NCCL_IB_DISABLE="1")


def rank_main():
    import numpy as np
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    from rpkt_amd import dist as rd, engine, gen
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    t0 = time.time()
    dist.init_process_group("nccl", device_id=torch.device("cuda", 0))
    n, nb = 400000, 8192
    lo, hi = rd.shard_range(n, rank, world)
    hb = gen.make_batch(4, hi - lo, first=lo)
    db = engine.DeviceBatch.from_host(hb)
    _, ev = engine.parse_batch(db, 3 | 4, n_buckets=nb)
    c = engine.flow_count(ev, hb.n, nb)
    out = {"rank": rank, "init_s": round(time.time() - t0, 2)}
    fail = int(os.environ.get("RPKT_PROBE_FAIL_RANK", "-1"))
    rd.COMM_INIT_TIMEOUT_MS = int(os.environ.get("RPKT_PROBE_TIMEOUT_MS", rd.COMM_INIT_TIMEOUT_MS))
    if rank == fail:
        def no_join(*a, **k):
            raise RuntimeError("probe: this rank fails before joining")
        engine.comm_init_timeout = no_join
    for via in ("auto", "own"):
        x = c.clone()
        t1 = time.time()
        rd.reduce_counters(x, n_buckets=nb, via=via)
        torch.cuda.synchronize()
        out[via] = {"path": rd.last_reduce_path, "error": rd.last_reduce_error,
                    "pkts": int(rd.counters_as_u64(x)[:, 0].sum()),
                    "seconds": round(time.time() - t1, 2)}
        ref = c.clone()
        rd.reduce_counters(ref, via="torch")
        out[via]["equal_torch"] = bool(torch.equal(ref, x))
    dist.barrier()
    rd.release_own_comms()
    dist.destroy_process_group()
    # one write(2) per rank: print() may issue the line and its newline as two writes
    # (unbuffered stdout), and the ranks share the pipe
    os.write(1, (json.dumps(out) + "\n").encode())


def main(world):
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = [subprocess.Popen([sys.executable, os.path.abspath(__file__), "--rank"],
                              env=share_env(r, world, port)) for r in range(world)]
    rc, t_end = 0, time.time() + 150
    try:
        for p in procs:
            rc = rc or p.wait(timeout=max(1.0, t_end - time.time()))
    except subprocess.TimeoutExpired:
        print(json.dumps({"error": "ranks still running after 150 s: killed"}), flush=True)
        rc = 124
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    sys.exit(rc)


if __name__ == "__main__":
    if "--rank" in sys.argv:
        rank_main()
    else:
        main(int(sys.argv[1]) if len(sys.argv) > 1 else 2)
