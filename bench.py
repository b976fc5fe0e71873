#!/usr/bin/env python3
"""bench.py — device-resident Ether/IPv4/{TCP,UDP} parse + checksum throughput.

Metric (BASELINE.json): Mpps + GB/s device-resident parse+cksum, 64 B & 1500 B
frames, 1/2/4/8 MI355X.  One "step" = one rpkt_gpu_parse_batch launch over one
synthetic batch already resident in HBM.

  headline  config 2: 1,048,576 x 64 B Ether/IPv4/UDP, stride 64, header extract +
            IPv4 header sum.  Each rank rotates over 8 distinct batches, so the frames
            alone (512 MiB, plus 640 MiB of records) are twice the 256 MiB Infinity
            Cache and every launch streams its frames from HBM.
  also      config 3: 1,048,576 x 1500 B Ether/IPv4/TCP, full L3 + L4 sums
            (reported under "extra").
  --config 4: 8,388,608-frame IMIX sharded over the ranks (strong scaling) with
            per-flow counters and one RCCL all-reduce of the counters.
  --config 7: 262,144 x 8000 B jumbo frames as mbuf chains (2048-B segments in
            shuffled 2176-B mempool slots), rpkt_gpu_parse_chains, full L3 + L4 sums.
  --config 10 / 11: dual stack (RPKT_F_IPV6), 1,048,576 x 64 B IPv4/UDP + IPv6/UDP and
            1,048,576 x 1500 B IPv4 + IPv6 (0-3 extension headers) TCP/UDP, full sums.

  config 1: benches/rpkt's packet_l4 over 1,000 x 64 B frames on the host CPU
            (oracle restatement, 1 thread), ns/pkt under "extra".

Multi-GPU: one process per GPU.  Under torchrun (WORLD_SIZE set) this process is one
rank; otherwise `--gpus N` (N > 1) starts the N rank processes itself, before any GPU
call, and exits with their status.  Batches are independent, so ranks never exchange
frames (weak scaling for configs 2/3); config 4 shards one batch and sums its flow
counters with rpkt_gpu_flow_reduce (RCCL).  The timed region is bracketed by
barrier + synchronize and the max over ranks is reported.  At N > 1 the default legs are
the headline, config 4 and the strong-scaling legs only (LEG_DEFAULTS, --all-legs).

Output: rank 0 prints ONE compact JSON line (< 8,000 bytes: the contract keys, the main
leg's roofline and CPU baseline, per extra leg its kernel/step times, roofline fraction
and traffic ratio) and writes every leg's full result to --detail
(gpurun_out/bench_detail.json), whose path the line gives.
"""
import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from rpkt_amd import dist as rdist, engine, fields, gen  # noqa: E402
from rpkt_amd.records import (as_tunnels, LAYERS_DTYPE, REC_BYTES, REC16_BYTES, F_FLOW_EV, F_IPV6,  # noqa: E402
                              as_records, is_ip6)

METRIC = "Mpps + GB/s device-resident parse+cksum, 64B & 1500B pkts, 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FLAG_NAMES = {1: "ip_sum", 2: "l4_sum", 3: "ip_sum+l4_sum", 11: "ip_sum+l4_sum+ipv6"}
WORKLOAD = {2: "1M x 64B Ether/IPv4/UDP extract + IPv4 header checksum",
            3: "1M x 1500B Ether/IPv4/TCP parse + full L3/L4 checksum",
            4: "8M IMIX 64/570/1500 (7:4:1) TCP/UDP, sharded, flow counters + RCCL reduce",
            5: "4M x U[64,1518]B 802.1Q/QinQ + IPv4 options -> TCP options",
            7: "256K x 8000B jumbo TCP/UDP as 2048-B mbuf chains, parse + full L3/L4 checksum",
            10: "1M x 64B dual stack IPv4/UDP + IPv6/UDP parse + full L3/L4 checksum",
            11: "1M x 1500B dual stack IPv4 + IPv6 (0-3 extension headers) TCP/UDP, full "
                "L3/L4 checksum"}


def log(rank, *a):
    if rank == 0:
        print("[bench]", *a, file=sys.stderr, flush=True)


def dist_env():
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    return rank, local, world


def barrier(world):
    if world > 1:
        dist.barrier()


def _red_device():
    return "cuda" if dist.get_backend() == "nccl" else "cpu"


def max_over_ranks(x, world):
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=_red_device())
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(x, world):
    if world == 1:
        return x
    t = torch.tensor([x], dtype=torch.float64, device=_red_device())
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def agree_all(ok, world):
    """True on every rank iff ok on every rank."""
    return ok if world == 1 else rdist.agree(ok)


def usable_cpus():
    """Host threads this process may run on: the affinity mask, capped by a cgroup v2
    CPU quota when one is set (a GPU box grants a share of a larger machine)."""
    n = len(os.sched_getaffinity(0))
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            quota, period = fh.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(quota) // int(period)))
    except (OSError, ValueError):
        pass
    return n


def share_gpu_env(rank):
    """--share-gpu: RCCL refuses two ranks of one host on one device ("Duplicate GPU
    detected"); a distinct NCCL_HOSTID per rank makes the ranks look like separate hosts,
    which then talk over the socket transport on loopback.  A one-GPU rehearsal of the
    cross-rank RCCL code (communicators, the C ABI all-reduce, torch's ProcessGroupNCCL),
    not an xGMI measurement."""
    return {"NCCL_HOSTID": "rpkt-share-%d" % rank, "NCCL_SOCKET_IFNAME": "lo",
            "NCCL_IB_DISABLE": "1"}


def launch_ranks(n, argv, share=False):
    """Start n rank processes of this script (RANK/LOCAL_RANK/WORLD_SIZE + a local
    rendezvous), wait for all of them and return the worst exit status.  Runs before
    anything touches the GPU; the ranks are children, never an exec of this process."""
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        if share:
            env.update(share_gpu_env(r))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv,
                                      env=env))
    rc = 0
    try:
        while procs:
            for p in list(procs):
                c = p.poll()
                if c is None:
                    continue
                procs.remove(p)
                if c != 0:
                    rc = rc or c
                    for q in procs:                 # one rank failed: the rest would hang
                        q.terminate()
            time.sleep(0.2)
    finally:
        for p in procs:
            p.kill()
    return rc


def algorithmic_bytes(hb, flow=False, rec_bytes=REC_BYTES):
    """Bytes one step must move: every frame byte read + the record written (80 B, or
    16 B compact) (+ 4 B offset per frame for the packed layout; + 8 B flow event
    written and read back by the flow-counter pass).  SURVEY.md §8d."""
    b = int(hb.lens().sum()) + hb.n * rec_bytes
    if isinstance(hb, gen.HostChains):             # segment descriptors + chain index
        return b + 8 * hb.n_segs + 4 * (hb.n + 1)
    if hb.offsets is not None:
        b += 4 * (hb.n + 1)
    if flow:
        b += 16 * hb.n
    return b


def time_parse(dbs, recs, flags, steps, warmup, world, flow=None, min_warm_s=0.3,
               compact=False, opts=None):
    """Time `steps` launches (rotating over dbs).  Returns wall seconds (max over
    ranks) and the mean per-launch device time from two HIP events recorded on the
    launch stream around the back-to-back launches."""
    stream = torch.cuda.current_stream()
    R = len(dbs)
    nb = flow["n_buckets"] if flow else 0

    def one(k):
        db, rc = dbs[k % R], recs[k % R]
        if flow:
            engine.parse_batch(db, flags | F_FLOW_EV, recs=rc, flow_ev=flow["ev"][k % R],
                               n_buckets=nb, stream=stream)
            engine.flow_count(flow["ev"][k % R], db.n, nb, counters=flow["counters"],
                              workspace=flow["ws"], stream=stream)
        elif opts is not None:                         # parse + option walks, one pass
            engine.parse_options_batch(db, flags, recs=rc, opts=opts[k % R], stream=stream,
                                       compact=compact)
        elif isinstance(db, engine.DeviceChains):
            engine.parse_chains(db, flags, recs=rc, stream=stream)
        elif compact:
            engine.parse_batch_compact(db, flags, recs=rc, stream=stream)
        else:
            engine.parse_batch(db, flags, recs=rc, stream=stream)

    # W untimed warmup launches, extended to >= min_warm_s of GPU work: after the
    # host-side batch generation the GPU sits idle and its clocks ramp back up over
    # tens of ms (measured: 339 us/launch over 20 steps vs 299 over 200 at 1500 B)
    k = 0
    t_w = time.perf_counter()
    while k < warmup or time.perf_counter() - t_w < min_warm_s:
        one(k)
        k += 1
        if k % 16 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    warm_launches = k
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev0.record(stream)
    for k in range(steps):
        one(k)
    ev1.record(stream)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier(world)
    wall = max_over_ranks(t1 - t0, world)
    kern_ms = ev0.elapsed_time(ev1) / steps      # back-to-back launches on `stream`
    return wall, kern_ms, warm_launches


def fused_vs_parse(dbs, recs, obufs, flags, compact, rounds=7, k=10):
    """The fused pass against the parse alone on the same batches, timed interleaved
    (k launches of each per round, HIP events on the launch stream; medians): the
    ratio does not move with the box's clocks as two legs timed minutes apart do."""
    stream = torch.cuda.current_stream()
    R = len(dbs)
    parse = engine.parse_batch_compact if compact else engine.parse_batch
    legs = {
        "parse": lambda j: parse(dbs[j % R], flags, recs=recs[j % R], stream=stream),
        "fused": lambda j: engine.parse_options_batch(dbs[j % R], flags, recs=recs[j % R],
                                                      opts=obufs[j % R], stream=stream,
                                                      compact=compact),
    }
    t = {name: [] for name in legs}
    for r in range(rounds + 1):                     # round 0 warms both
        for name, fn in legs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for j in range(k):
                fn(j)
            e1.record(stream)
            torch.cuda.synchronize()
            if r:
                t[name].append(e0.elapsed_time(e1) / k)
    med = {name: sorted(v)[len(v) // 2] for name, v in t.items()}
    return {"parse_kernel_ms": round(med["parse"], 5), "fused_kernel_ms": round(med["fused"], 5),
            "ratio": round(med["fused"] / med["parse"], 4), "rounds": rounds, "launches": k}


def pmc_traffic(cfg, compact=False, opts=False, n=None):
    """Per-launch HBM traffic of parse_kernel for this config (and record size, and the
    fused option walks) from the rocprofv3 PMC summary committed under profiles/
    (tools/traffic.py), when it was measured on this exact engine build and a launch
    covers as many frames as the profiled one; else None."""
    if n is not None and not profiled_size(cfg, n):
        return None, None
    path = os.path.join(ROOT, "profiles", "traffic_c%d%s%s.json" % (
        cfg, "_opts" if opts else "", "_compact" if compact else ""))
    try:
        with open(path) as fh:
            t = json.load(fh)
    except (OSError, ValueError):
        return None, None
    if not same_unit(t.get("engine_build"), "parse"):
        return None, None
    return int(t["traffic_bytes_per_launch"]), os.path.relpath(path, ROOT)


def profiled_size(cfg, n):
    """Whether a launch over n frames of config cfg matches the committed PMC profiles:
    they are taken by scripts/refresh_profiles.sh at N=1 with the default frame counts, so
    an N-rank shard (config 4, the strong legs) or a --frames run gets traffic None."""
    return n == gen.DEFAULT_N[cfg]


def same_unit(profiled_build, unit):
    """Whether a profile taken on engine build `profiled_build` measured the same source
    of kernel unit `unit` (rpkt_<unit>.hip + the shared headers) as the loaded build."""
    def unit_hash(b):
        for tok in (b or "").replace(";", " ").split():
            if tok.startswith(unit + "="):
                return tok
        return None
    cur = engine.lib().rpkt_gpu_build_info().decode()
    if profiled_build == cur:
        return True
    h = unit_hash(cur)
    return h is not None and h == unit_hash(profiled_build)


def pmc_traffic_tx(leg, n=None):
    """Per-launch HBM traffic of a TX / walk leg (profiles/traffic_tx.json, from a
    rocprofv3 PMC profile of those legs on this exact engine build, at the profiled frame
    count); else None."""
    if n is not None and not profiled_size(int(leg.lstrip("abcdefghijklmnopqrstuvwxyz")), n):
        return None, None
    path = os.path.join(ROOT, "profiles", "traffic_tx.json")
    try:
        with open(path) as fh:
            t = json.load(fh)
    except (OSError, ValueError):
        return None, None
    unit = {"build": "tx", "forward": "tx", "opts": "walks", "optsc": "walks", "layers": "walks",
            "fields": "fields", "tunnel": "tunnel", "encap": "tx"}[leg.rstrip("0123456789")]
    if leg not in t["legs"] or not same_unit(t["legs"][leg].get("engine_build", t.get("engine_build")),
                                             unit):
        return None, None
    return int(t["legs"][leg]["traffic_bytes_per_launch"]), os.path.relpath(path, ROOT)


def head_sample(hb, max_bytes=256 << 20):
    """The first frames of a host batch, at most ~max_bytes of frame data."""
    lens = hb.lens()
    m = int(np.searchsorted(np.cumsum(lens), max_bytes)) if lens.sum() > max_bytes else hb.n
    m = max(1, min(m, hb.n))
    if hb.offsets is not None:
        offs = hb.offsets[:m + 1]
        return gen.HostBatch(hb.config, m, hb.seed, hb.frames[:int(offs[-1])], offs, 0, 0)
    return gen.HostBatch(hb.config, m, hb.seed, hb.frames[:m * hb.stride], None, hb.stride,
                         hb.frame_len)


def cpu_model():
    """The host CPU's model name (SURVEY.md §8d asks for it beside the core count)."""
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


_ORACLE_BUILD = None


def oracle_for_baseline():
    """The oracle, loaded from an -O3 -march=native build made on this host when gcc
    is available, else from the shipped -march=x86-64-v3 build."""
    global _ORACLE_BUILD
    from oracle import oracle
    if _ORACLE_BUILD is None:
        _ORACLE_BUILD = oracle.use_native_build() or "-O3 -march=x86-64-v3 (shipped build)"
    return oracle, _ORACLE_BUILD


def timed_reps(fn, seconds):
    """Run fn() once (cold: caches, page faults), then repeat it until >= `seconds` have
    passed; returns (reps, elapsed)."""
    fn()
    reps, t0 = 0, time.perf_counter()
    while True:
        fn()
        reps += 1
        dt = time.perf_counter() - t0
        if dt >= seconds:
            return reps, dt


def cpu_fields(value_mpps, gbs, threads, sample, reps, dt, build):
    return {"value": round(value_mpps, 3), "unit": "Mpps", "cores": threads,
            "gb_per_s": round(gbs, 3), "reps": reps, "seconds": round(dt, 2),
            "sample": sample, "build": build}


def flatten_all_cores(out):
    """SURVEY.md §8(d)(ii), the all-host-cores baseline, as scalars beside the 1-thread
    value (records that keep only the top level of cpu_baseline still carry it)."""
    a = out["all_cores"]
    out.update(all_cores_mpps=a["value"], all_cores_gb_per_s=a["gb_per_s"],
               all_cores_threads=a["cores"],
               # all-threads rate over the 1-thread rate: how far the static partition scales
               all_cores_scaling=round(a["value"] / out["value"], 2) if out["value"] else None)
    return out


def cpu_baseline_chains(hc, gpu_recs, flags, seconds, threads_all, max_bytes=256 << 20):
    """Chain oracle (oracle/rpkt_oracle_chain.c) over the first chains of the batch
    (~max_bytes of frame data), 1 thread and all usable host threads, each for
    >= `seconds`; checks the GPU records of the sample."""
    oracle, build = oracle_for_baseline()
    m = int(np.searchsorted(np.cumsum(hc.lens()), max_bytes))
    m = max(1, min(m, hc.n))
    first = hc.chain_first[:m + 1]
    segs = hc.segs[:int(first[-1])]
    o = oracle.parse_chains(hc.buf, segs, first, flags)
    nbytes = int(hc.lens()[:m].sum())
    sample = "first %d chains (%.0f MB, %d segments) of the batch" % (m, nbytes / 1e6,
                                                                       segs.shape[0])
    # the record buffer is allocated once, outside the timed reps (the reference's harness
    # allocates nothing per iteration, benches/rpkt/rpkt_parse.rs:108-140); timed_reps'
    # untimed first call first-touches each thread's slice of it
    out = np.empty_like(o)
    reps, dt = timed_reps(lambda: oracle.parse_chains(hc.buf, segs, first, flags, out=out), seconds)
    reps_a, dt_a = timed_reps(lambda: oracle.parse_chains(hc.buf, segs, first, flags,
                                                          threads=threads_all, out=out), seconds)
    out = cpu_fields(m * reps / dt / 1e6, nbytes * reps / dt / 1e9, 1,
                     "%d reps x %s, 1 thread" % (reps, sample), reps, dt, build)
    out.update(kind="port", cpu_model=cpu_model(), host_logical_cpus=os.cpu_count(),
               all_cores=cpu_fields(m * reps_a / dt_a / 1e6, nbytes * reps_a / dt_a / 1e9,
                                    threads_all, "%d reps x %s, %d threads (static partition)"
                                    % (reps_a, sample, threads_all), reps_a, dt_a, build),
               gpu_parity_on_sample=bool(gpu_recs[:m].tobytes() == o.tobytes()))
    return flatten_all_cores(out)


def cpu_parse_callable(oracle, hb, flags, threads):
    """The timed body of the CPU baseline: the oracle's parse of the sample into a record
    buffer allocated here, once (the reference's criterion loop allocates nothing per
    iteration, benches/rpkt/rpkt_parse.rs:108-140).  timed_reps' untimed first call
    first-touches each thread's slice of it, so the timed calls measure the parse alone
    (tests/test_bench_cli.py checks that a call allocates nothing)."""
    from rpkt_amd.records import REC_DTYPE
    out = np.empty(hb.n, dtype=REC_DTYPE)
    frames = np.ascontiguousarray(hb.frames, dtype=np.uint8)
    offs = None if hb.offsets is None else np.ascontiguousarray(hb.offsets, dtype=np.uint32)

    def run():
        oracle.parse_batch(frames, hb.n, flags=flags, offsets=offs, stride=hb.stride,
                           frame_len=hb.frame_len, threads=threads, out=out)
    run.out = out
    return run


def cpu_baseline(hb, gpu_recs, flags, seconds, threads_all):
    """The CPU restatement of rpkt's path (oracle/, kind "port") timed on this host
    over a bounded sample of the same workload, 1 thread and all usable host threads,
    each for >= `seconds`; also checks the GPU records of the sample bit-exact."""
    oracle, build = oracle_for_baseline()
    hb = head_sample(hb)
    gpu_recs = gpu_recs[:hb.n]
    n = hb.n
    nbytes = int(hb.lens().sum())

    o = oracle.parse_batch(hb.frames, n, flags=flags, offsets=hb.offsets, stride=hb.stride,
                           frame_len=hb.frame_len)
    sample = "first %d frames (%.0f MB) of the batch" % (n, nbytes / 1e6)
    reps, dt = timed_reps(cpu_parse_callable(oracle, hb, flags, 1), seconds)
    reps_a, dt_a = timed_reps(cpu_parse_callable(oracle, hb, flags, threads_all), seconds)
    out = cpu_fields(n * reps / dt / 1e6, nbytes * reps / dt / 1e9, 1,
                     "%d reps x %s, 1 thread" % (reps, sample), reps, dt, build)
    out.update(kind="port", cpu_model=cpu_model(), host_logical_cpus=os.cpu_count(),
               all_cores=cpu_fields(n * reps_a / dt_a / 1e6, nbytes * reps_a / dt_a / 1e9,
                                    threads_all, "%d reps x %s, %d threads (static partition)"
                                    % (reps_a, sample, threads_all), reps_a, dt_a, build),
               gpu_parity_on_sample=bool(gpu_recs.tobytes() == o.tobytes()))
    return flatten_all_cores(out)


def run_config1(args):
    """Config 1 (BASELINE.json configs[0]): benches/rpkt's `packet_l4`
    (rpkt_parse.rs:62-80) over 1,000 x 64 B Ether/IPv4/UDP frames built like
    rpkt_build.rs:13-27, the oracle restatement on 1 host thread, >= cpu_seconds.
    Reported in ns/pkt and Mpps like criterion would."""
    oracle, build = oracle_for_baseline()
    hb = gen.make_batch(1)
    r = oracle.parse_batch(hb.frames, hb.n, flags=3, stride=hb.stride)
    keys = ("ip_src", "ip_dst", "ip_checksum", "ip_ident", "src_port", "dst_port",
            "l4_word6", "l4_checksum")
    want = tuple(int(r[k][0]) for k in keys)
    flen = hb.frame_len or hb.stride
    bad = oracle.packet_l4_loop(hb.frames, hb.n, hb.stride, flen, 1, want)
    reps_probe = 1000
    t0 = time.perf_counter()
    oracle.packet_l4_loop(hb.frames, hb.n, hb.stride, flen, reps_probe, want)
    one = (time.perf_counter() - t0) / reps_probe
    reps = max(1, int(args.cpu_seconds / max(one, 1e-9)))
    t0 = time.perf_counter()
    bad += oracle.packet_l4_loop(hb.frames, hb.n, hb.stride, flen, reps, want)
    dt = time.perf_counter() - t0
    ns = dt / (reps * hb.n) * 1e9
    # the same loop on every usable host thread at once: each thread
    # makes reps_a passes over the 1,000 frames
    threads = max(1, args.cpu_threads or usable_cpus())
    reps_a = max(1, reps // 2)
    t0 = time.perf_counter()
    bad += oracle.packet_l4_loop_mt(hb.frames, hb.n, hb.stride, flen, reps_a, want, threads)
    dt_a = time.perf_counter() - t0
    mpps_a = threads * reps_a * hb.n / dt_a / 1e6
    return {"ns_per_pkt": round(ns, 3), "mpps": round(1e3 / ns, 2), "cores": 1,
            "frames": hb.n, "frame_bytes": 64, "reps": reps, "seconds": round(dt, 2),
            "all_cores_mpps": round(mpps_a, 2), "all_cores_threads": threads,
            "all_cores_seconds": round(dt_a, 2),
            "all_cores_scaling": round(mpps_a / (1e3 / ns), 2),
            "asserts_failed": bad, "kind": "port", "build": build, "cpu_model": cpu_model(),
            "what": "benches/rpkt packet_l4 (rpkt_parse.rs:62-80) restated in C, per frame"}


def layout_name(hb):
    if isinstance(hb, gen.HostChains):
        return "mbuf chains: %d segments of <= %d B, shuffled %d-B slots" % (
            hb.n_segs, gen.MBUF_ROOM, gen.MBUF_ROOM + gen.MBUF_HEADROOM)
    return ("stride%d" % hb.stride) if hb.stride else "packed+u32 offsets"


def run_config(cfg, args, rank, world, cpu=False, compact=False, opts=False, strong=False,
               main=False):
    """One parse leg: config `cfg`'s batches resident, K timed launches.  compact: the
    16-byte record entry point (rpkt_gpu_parse_batch_compact) instead of the 80-byte one.
    opts: the fused parse + option walks (rpkt_gpu_parse_options_batch[_compact]), 64 B
    more written per frame.  strong: configs 2/3 as one batch split over the ranks
    (rdist.shard_range), each rank rotating over enough distinct batches that its shards
    outgrow the 256 MiB Infinity Cache twice over."""
    flags = gen.FLAGS[cfg]
    flow = None
    if cfg == 4:                                   # strong scaling: shard one 8M batch
        n_total = args.frames or gen.DEFAULT_N[4]
        lo, hi = rdist.shard_range(n_total, rank, world)
        hbs = [gen.make_batch(4, hi - lo, first=lo)]
        scaling = "strong"
    elif strong:                                   # strong scaling: shard one batch
        n_total = args.frames or gen.DEFAULT_N[cfg]
        lo, hi = rdist.shard_range(n_total, rank, world)
        shard_bytes = max(1, (hi - lo) * gen.STRIDED.get(cfg, 1024))
        R = max(8 if cfg == 2 else 1, -(-(512 << 20) // shard_bytes))
        hbs = [gen.make_batch(cfg, hi - lo, seed=gen.DEFAULT_SEED[cfg] + 104729 * r, first=lo)
               for r in range(R)]
        scaling = "strong"
    elif cfg in gen.CHAINED:                       # weak scaling: chains per rank
        n = args.frames or gen.DEFAULT_N[cfg]
        hbs = [gen.make_chains(cfg, n, seed=gen.DEFAULT_SEED[cfg] + 7919 * rank)]
        scaling = "weak"
    else:                                          # weak scaling: a batch per rank
        n = args.frames or gen.DEFAULT_N[cfg]
        R = args.rotate or (8 if cfg in (2, 10) else 1)
        hbs = [gen.make_batch(cfg, n, seed=gen.DEFAULT_SEED[cfg] + 7919 * rank + 104729 * r)
               for r in range(R)]
        scaling = "weak"
    dbs = [engine.DeviceChains.from_host(hb) if cfg in gen.CHAINED else
           engine.DeviceBatch.from_host(hb) for hb in hbs]
    rec_bytes = REC16_BYTES if compact else REC_BYTES
    recs = [torch.empty(hb.n * rec_bytes, dtype=torch.uint8, device="cuda") for hb in hbs]
    obufs = [torch.empty(hb.n * 64, dtype=torch.uint8, device="cuda") for hb in hbs] if opts else None
    if cfg == 4:
        nb = 8192
        flow = {"n_buckets": nb,
                "ev": [torch.empty(hb.n, dtype=torch.int64, device="cuda") for hb in hbs],
                "counters": torch.zeros((nb + 1) * 4, dtype=torch.int64, device="cuda"),
                "ws": engine.flow_workspace(hbs[0].n, nb)}
    torch.cuda.synchronize()
    log(rank, "config %d: %d frames/rank x %d batches resident, flags=%d" % (
        cfg, hbs[0].n, len(hbs), flags))
    wall, kern_ms, warm = time_parse(dbs, recs, flags, args.steps, args.warmup, world, flow,
                                     args.min_warmup_s, compact, obufs)

    frames_step = sum(hb.n for hb in hbs) / len(hbs)
    bytes_step = sum(int(hb.lens().sum()) for hb in hbs) / len(hbs)
    alg_step = sum(algorithmic_bytes(hb, flow is not None, rec_bytes + (64 if opts else 0))
                   for hb in hbs) / len(hbs)
    # whole-job frames per step: every rank's shard (they differ by at most one frame)
    frames_job = sum_over_ranks(frames_step, world) if scaling == "strong" else frames_step * world
    bytes_job = sum_over_ranks(bytes_step, world) if scaling == "strong" else bytes_step * world
    mpps = frames_job * args.steps / wall / 1e6
    gbps = bytes_job * args.steps / wall / 1e9
    achieved = alg_step / (kern_ms / 1e3) / 1e9
    # N > 1: every rank's achieved GB/s summed (each rank has its own HBM), beside the
    # per-rank fraction `frac` (a collective: every rank calls it)
    achieved_all = sum_over_ranks(achieved, world) if world > 1 else None
    traffic, tsrc = pmc_traffic(cfg, compact, opts, hbs[0].n)
    out = {
        "mpps": mpps, "frame_gb_per_s": gbps, "ms_per_step": wall / args.steps * 1e3,
        "warmup_launches": warm,
        "kernel_ms": kern_ms, "scaling": scaling, "frames_per_rank": int(frames_step),
        "frames_per_step": int(frames_job), "batches_rotated": len(hbs),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "traffic_source": tsrc,
                     "alg_bytes_per_launch": int(alg_step)},
        "flags": FLAG_NAMES[flags], "layout": layout_name(hbs[0]),
        "record_bytes": rec_bytes,
    }
    if achieved_all is not None:
        out["roofline"].update(achieved_all_ranks=round(achieved_all, 1),
                               peak_all_ranks=HBM_PEAK_GBS * world)
    if compact:
        out["what"] = ("rpkt_gpu_parse_batch_compact: the same parse + sums, 16-B records "
                       "(status, offsets, sums, verdicts)")
    if opts:
        out["what"] = ("rpkt_gpu_parse_options_batch%s: the parse + sums and both option walks "
                       "(Ipv4OptionsIter, TcpOptionsIter) in one pass, 64-B rpkt_opts_t per frame"
                       % ("_compact" if compact else ""))
        out["vs_parse_same_run"] = fused_vs_parse(dbs, recs, obufs, flags, compact)
    if cfg == 4:
        torch.cuda.synchronize()
        barrier(world)
        # the per-rank counters, kept to check the product reduce against torch's own
        local = flow["counters"].clone() if world > 1 else None
        # one untimed reduce of a zero buffer first: the communicator's creation (own: rank
        # 0's id broadcast + ncclCommInitRank) and RCCL's first-collective connection setup
        # are paid once per job, not by the reduce the line reports
        zeros = torch.zeros_like(flow["counters"])
        rdist.reduce_counters(zeros, n_buckets=nb, via=args.reduce_comm)
        torch.cuda.synchronize()
        barrier(world)
        # the reduce time: REDUCE_SAMPLES reduces of a scratch copy (each one sums in place,
        # so the real counters are reduced once, below), each bracketed by a barrier and a
        # synchronize, the max over ranks per sample; median, min and max reported (one
        # latency-bound 262-KB all-reduce is too short for a single sample to mean much)
        scratch = flow["counters"].clone()
        samples = []
        for _ in range(REDUCE_SAMPLES):
            torch.cuda.synchronize()
            barrier(world)
            t0 = time.perf_counter()
            rdist.reduce_counters(scratch, n_buckets=nb, via=args.reduce_comm)
            torch.cuda.synchronize()
            samples.append(max_over_ranks(time.perf_counter() - t0, world) * 1e3)
        del scratch
        torch.cuda.synchronize()
        barrier(world)
        # rpkt_gpu_flow_reduce (RCCL, C ABI) when every rank can call it, else torch's
        # all-reduce on every rank; a failure after the group chose the C ABI raises
        rdist.reduce_counters(flow["counters"], n_buckets=nb, via=args.reduce_comm)
        torch.cuda.synchronize()
        c = rdist.counters_as_u64(flow["counters"])
        out["flow_reduce_ms"] = float(np.median(samples))
        out["flow_reduce_ms_min"] = min(samples)
        out["flow_reduce_ms_max"] = max(samples)
        out["flow_reduce_samples"] = len(samples)
        out["flow_reduce_via"] = rdist.last_reduce_path
        if rdist.last_reduce_error:
            out["flow_reduce_error"] = "C ABI reduce not taken: %s" % rdist.last_reduce_error
        if local is not None:                        # every word vs torch.distributed's sum
            rdist.reduce_counters(local, via="torch")
            same = torch.equal(local, flow["counters"])
            out["flow_reduce_verified"] = bool(agree_all(same, world))
            if not out["flow_reduce_verified"]:
                out["flow_reduce_error"] = ("reduced counters differ from torch.distributed's "
                                            "all_reduce of the same per-rank counters")
        out["flow_pkts_total"] = int(c[:, 0].sum())
        # every launch (warmup included) added its shard's frames to the counters
        out["flow_pkts_expected"] = int(sum_over_ranks(hbs[0].n * (args.steps + warm), world))
    # the records of batch 0 are read back before the copy references overwrite them
    g = as_records(recs[0].cpu().numpy()) if cpu and rank == 0 and not compact and not opts \
        else None
    if cfg == 2 and main and not compact and not strong and world == 1:
        try:
            out["copy_ceiling"] = copy_ceiling(dbs, recs, args.steps)
        except engine.RpktError as e:           # the development library is optional
            out["copy_ceiling"] = {"error": str(e)}
    if g is not None:
        if cfg in gen.CHAINED:
            out["cpu_baseline"] = cpu_baseline_chains(hbs[0], g, flags, args.cpu_seconds,
                                                      args.cpu_threads)
        else:
            out["cpu_baseline"] = cpu_baseline(hbs[0], g, flags, args.cpu_seconds,
                                               args.cpu_threads)
    del dbs, recs
    torch.cuda.empty_cache()
    return out


def run_ring(cfg, args, rank, world, slots=8, compact=False):
    """A receive ring of `slots` full-size batches of config `cfg` (8 x 1M x 64 B for
    config 2) parsed by ONE rpkt_gpu_parse_ring[_compact] launch per step: the batch
    boundary's fixed cost (launch, first-round ramp, last-round drain) is paid once per
    8M frames instead of once per 1M.  Same batches, flags and records as the headline
    leg, which parses them one launch per batch."""
    n = args.frames or gen.DEFAULT_N[cfg]
    flags = gen.FLAGS[cfg]
    hbs = [gen.make_batch(cfg, n, seed=gen.DEFAULT_SEED[cfg] + 7919 * rank + 104729 * r)
           for r in range(slots)]
    dbs = [engine.DeviceBatch.from_host(hb) for hb in hbs]
    rec_bytes = REC16_BYTES if compact else REC_BYTES
    recs = [torch.empty(hb.n * rec_bytes, dtype=torch.uint8, device="cuda") for hb in hbs]
    ring = engine.ring_slots(dbs, recs, compact=compact)
    stream = torch.cuda.current_stream()

    def one():
        engine.parse_ring(ring, flags, 0, stream=stream, compact=compact)
    k, t_w = 0, time.perf_counter()
    while k < args.warmup or time.perf_counter() - t_w < args.min_warmup_s:
        one()
        k += 1
        if k % 4 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    steps = max(4, args.steps // slots)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier(world)
    t0 = time.perf_counter()
    ev0.record(stream)
    for _ in range(steps):
        one()
    ev1.record(stream)
    torch.cuda.synchronize()
    wall = max_over_ranks(time.perf_counter() - t0, world)
    kern_ms = ev0.elapsed_time(ev1) / steps
    frames = sum(hb.n for hb in hbs)
    alg = sum(algorithmic_bytes(hb, rec_bytes=rec_bytes) for hb in hbs)
    achieved = alg / (kern_ms / 1e3) / 1e9
    out = {"mpps": frames * world * steps / wall / 1e6, "kernel_ms": kern_ms,
           "ms_per_step": wall / steps * 1e3, "frames_per_launch": frames, "slots": slots,
           "launches": steps, "record_bytes": rec_bytes, "flags": FLAG_NAMES[flags],
           "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                        "alg_bytes_per_launch": int(alg)},
           "what": "rpkt_gpu_parse_ring%s: %d slots of %d frames in one launch" % (
               "_compact" if compact else "", slots, n)}
    del dbs, recs, ring
    torch.cuda.empty_cache()
    return out


# host-inclusive pipeline shape per config: device slots and 1M-frame batches per copy
# (tools/host_rate.py sweeps them; profiles/r03_host/)
HOST_SHAPE = {2: (3, 4), 3: (3, 1), 4: (3, 1)}


def run_host(args):
    """The path from and to host memory (north_star): pinned
    hipMemcpyAsync H2D of the frames, the parse, D2H of the records, pipelined on three
    streams (rpkt_amd.pipeline), with 80-B and 16-B records.  PCIe-bound; never the
    headline value."""
    from rpkt_amd import pipeline
    out = {}
    for c in [int(x) for x in args.host.split(",") if x.strip()]:
        slots, group = HOST_SHAPE.get(c, (3, 1))
        for compact in (False, True):
            r = pipeline.host_inclusive(c, compact, slots=slots, group=group)
            out["config%d%s" % (c, "_compact" if compact else "")] = {
                k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items()}
            torch.cuda.empty_cache()
    return out


def run_rx_graph(args):
    """A receive loop of small batches (rpkt_amd.graphs): a ring of `slots` batches of
    config-2 frames; per pass, each slot's parse with flow events and one flow count of
    the pass's events.  Timed as eager engine calls from Python (each through ctypes) and
    as one captured hipGraph replayed per pass, with the parses on the current stream,
    forked over 4 streams, or all slots in one rpkt_gpu_parse_ring call.  Every mode must
    leave identical counters."""
    from rpkt_amd import graphs
    out = {}
    nb = 1024
    for spec in [x for x in args.rx_graph.split(",") if x.strip()]:
        n, slots = (int(v) for v in spec.split("x"))
        hb = gen.make_batch(2, n, seed=gen.DEFAULT_SEED[2])
        ring = graphs.batch_ring(hb, slots)
        recs = [engine.alloc_records(n) for _ in range(slots)]
        ev_all = torch.empty(n * slots, dtype=torch.int64, device="cuda")
        ws = engine.flow_workspace(n * slots, nb)
        side = [torch.cuda.Stream() for _ in range(4)]
        evs = [ev_all[k * n:(k + 1) * n] for k in range(slots)]
        rslots = engine.ring_slots(ring, recs, evs)
        recs16 = [torch.empty(n * REC16_BYTES, dtype=torch.uint8, device="cuda") for _ in range(slots)]
        rslots16 = engine.ring_slots(ring, recs16, evs)
        res, cnts = {}, []
        for mode in ("eager", "graph", "eager_4streams", "graph_4streams", "ring", "ring_graph",
                     "ring_compact"):
            cnt = torch.zeros((nb + 1) * 4, dtype=torch.int64, device="cuda")
            cnts.append(cnt)
            streams = side if mode.endswith("4streams") else None
            if mode == "ring_compact":
                fn = (lambda cnt=cnt: graphs.rx_pass_ring(rslots16, ev_all, n * slots, cnt, ws,
                                                          gen.FLAGS[2], nb, compact=True))
            elif mode.startswith("ring"):
                fn = (lambda cnt=cnt: graphs.rx_pass_ring(rslots, ev_all, n * slots, cnt, ws,
                                                          gen.FLAGS[2], nb))
            else:
                fn = (lambda cnt=cnt, streams=streams:
                      graphs.rx_pass(ring, recs, ev_all, cnt, ws, gen.FLAGS[2], nb, streams))
            step = fn
            if mode.startswith("graph") or mode == "ring_graph":
                step = graphs.CapturedLoop(fn).replay      # runs one warm pass, then captures
            else:
                fn()                                       # the same warm pass
            for _ in range(3):
                step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                step()
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
            res[mode] = {"mpps": n * slots * args.steps / dt / 1e6,
                         "us_per_pass": dt / args.steps * 1e6}
        res["counters_identical"] = all(torch.equal(cnts[0], c) for c in cnts[1:])
        out["%dx%d" % (n, slots)] = {
            k: ({kk: round(vv, 3) for kk, vv in v.items()} if isinstance(v, dict) else v)
            for k, v in res.items()}
        del ring, recs, recs16, ev_all
        torch.cuda.empty_cache()
    return out


def copy_ceiling(dbs, recs, steps):
    """Measured device-to-device copy ceilings beside config 2, same
    stream and event timing as the parse (development library's streaming references):
      wave_mix / wave_mix_nt: wave-contiguous 16-B/lane streams of config 2's own bytes
        (the 8 rotated 64 MiB frame buffers read, 80 MiB of records written at the
        64 : 80 ratio throughout), default / non-temporal policy (variants 16 / 17);
      wave_copy / wave_copy_nt: the same kernel as a 1:1 memcpy of 1 GiB (18 / 19);
      same_mix_copy: the round-2 grid-stride copy of config 2's bytes (variant 13);
      d2d_memcpy: hipMemcpyAsync device to device of 1 GiB (torch copy_).
    Read + written bytes are counted."""
    L = engine.ablate_lib()               # the streaming references: development library
    L.rpkt_gpu_debug_variant.argtypes = [ctypes.POINTER(engine.Batch), ctypes.c_uint32,
                                         ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    L.rpkt_gpu_debug_variant.restype = ctypes.c_int
    stream = torch.cuda.current_stream()
    sp = ctypes.c_void_p(stream.cuda_stream)
    descs = [db.desc() for db in dbs]
    R = len(dbs)

    def timed(fn, k):
        for j in range(max(4, R)):
            fn(j)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for j in range(k):
            fn(j)
        e1.record(stream)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / k / 1e3                     # seconds per launch

    def variant(v, ds, outs):
        def run(j):
            rc = L.rpkt_gpu_debug_variant(ctypes.byref(ds[j % len(ds)]), 1,
                                          outs[j % len(outs)].data_ptr(), v, sp)
            if rc:
                raise engine.RpktError("copy reference %d: rc %d" % (v, rc))
        return run

    def entry(t, nbytes, what):
        return {"gb_per_s": round(nbytes / t / 1e9, 1), "us": round(t * 1e6, 2),
                "bytes": int(nbytes), "what": what}

    out = {}
    k = max(steps, 2 * R)
    mix_bytes = dbs[0].frames.numel() + recs[0].numel()
    mix_what = ("config 2's bytes: 64 MiB frames read, 80 MiB records written, 8 rotated "
                "batches, ")
    for name, v, what in (("wave_mix", 16, "wave-contiguous 16-B/lane, default policy"),
                          ("wave_mix_nt", 17, "wave-contiguous 16-B/lane, non-temporal"),
                          ("same_mix_copy", 13, "grid-stride copy (round 2's reference)")):
        out[name] = entry(timed(variant(v, descs, recs), k), mix_bytes, mix_what + what)
    a = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
    b = torch.empty_like(a)
    big = [engine.Batch(a.data_ptr(), a.numel(), None, 64, 64, 1, 0)]
    for name, v, what in (("wave_copy", 18, "default policy"), ("wave_copy_nt", 19, "non-temporal")):
        out[name] = entry(timed(variant(v, big, [b]), 10), 2 * (1 << 30),
                          "wave-contiguous 16-B/lane memcpy of 1 GiB (read + write), " + what)
    out["d2d_memcpy"] = entry(timed(lambda j: b.copy_(a), 10), 2 * (1 << 30),
                              "hipMemcpyAsync device to device, 1 GiB (read + write)")
    del a, b
    return out


FORBID_IPS = ["192.168.5.%d" % k for k in range(3, 11)]    # loopback_rx.rs:42-51


def line_floor(starts, ends, line=128):
    """Bytes of the distinct `line`-byte lines of the frame buffer that hold any byte of
    the ranges [starts, ends): the least a kernel reading exactly those bytes fetches,
    since every read request the memory side sends on gfx950 is a whole 128-B line
    (TCC_EA0_RDREQ_128B = all requests, profiles/r04_rdreq/)."""
    starts, ends = np.asarray(starts, np.int64), np.asarray(ends, np.int64)
    m = ends > starts
    a, b = starts[m] // line, (ends[m] - 1) // line
    if a.size == 0:
        return 0
    o = np.argsort(a, kind="stable")
    a, b = a[o], b[o]
    new = np.ones(a.size, bool)
    new[1:] = a[1:] > np.maximum.accumulate(b)[:-1]
    idx = np.flatnonzero(new)
    return int((np.maximum.reduceat(b, idx) - a[idx] + 1).sum()) * line


def ip_u32(s):
    a, b, c, d = (int(x) for x in s.split("."))
    return (a << 24) | (b << 16) | (c << 8) | d


# The fields leg's requests: the getters a receive loop reads on the capture mix.
FIELD_LEG = [("ETHER_ETHERFRAME", "dst_addr"), ("ETHER_ETHERFRAME", "src_addr"),
             ("ETHER_ETHERFRAME", "ethertype"), ("VLAN_VLANFRAME", "vlan_id"),
             ("IPV4_IPV4", "src_addr"), ("IPV4_IPV4", "dst_addr"), ("IPV4_IPV4", "ttl"),
             ("IPV4_IPV4", "protocol"), ("IPV6_IPV6", "src_addr", 0, "hi"),
             ("IPV6_IPV6", "src_addr", 0, "lo"), ("IPV6_IPV6", "flow_label"),
             ("IPV6_IPV6", "next_header"), ("UDP_UDP", "src_port"), ("UDP_UDP", "dst_port"),
             ("TCP_TCP", "seq_num"), ("VXLAN_VXLAN", "vni")]


TX_MODES = ("build", "forward", "opts", "optsc", "layers", "fields", "tunnel", "encap")


def tx_legs(spec):
    """--tx "build2,optsc5,..." -> [(leg, mode, config)]; an unknown leg is an error."""
    out = []
    for leg in [x.strip() for x in spec.split(",") if x.strip()]:
        mode = leg.rstrip("0123456789")
        if mode not in TX_MODES or mode == leg:
            raise SystemExit("bench.py: unknown --tx leg %r (modes %s + a config number)"
                             % (leg, ", ".join(TX_MODES)))
        out.append((leg, mode, int(leg[len(mode):])))
    return out


def run_tx(cfg, mode, args, rank, world):
    """TX side: rpkt_gpu_build_batch (headers + both checksums filled, the
    rpkt_build.rs path) or rpkt_gpu_forward_batch (loopback_rx rewrite) over a
    resident batch whose records come from rpkt_gpu_parse_batch.  Rotates over 8
    batches at 64 B like config 2.  Algorithmic bytes per frame: build = 80 B record
    read + the frame read once (checksums) + the fixed header bytes written;
    forward (fused parse + verdict + rewrite) = the frame read once + the rewritten
    header bytes of forwarded frames (0 .. l4 + 8: 42 B IPv4, 62 B IPv6) + 1 B verdict.
    Dual-stack configs (10, 11) parse with RPKT_F_IPV6: build writes IPv6 records too,
    forward passes RPKT_F_IPV6."""
    torch.cuda.empty_cache()
    n = args.frames or gen.DEFAULT_N[cfg]
    R = 8 if cfg == 2 else 1                  # 64-B legs: 512 MiB of frames, past the cache
    if cfg == 9:                                   # protocol mix (captures + fuzz)
        hbs = [gen.make_mix(n, seed=gen.DEFAULT_SEED[9] + 7919 * rank)]
    else:
        hbs = [gen.make_batch(cfg, n, seed=gen.DEFAULT_SEED[cfg] + 7919 * rank + 104729 * r)
               for r in range(R)]
    dbs = [engine.DeviceBatch.from_host(hb) for hb in hbs]
    pflags = gen.FLAGS.get(cfg, 3) | 3         # dual-stack configs: IPv6 records too
    fwd_flags = pflags & F_IPV6                # forward: IPv6 frames too (rpkt_fwd_t.flags)
    recs = [engine.parse_batch(db, pflags) for db in dbs]
    # optsc: the option walks located by compact records (rpkt_gpu_options_batch_compact)
    recs16 = [engine.parse_batch_compact(db, 3) for db in dbs] if mode == "optsc" else None
    outs = [torch.empty(hb.n * (64 if mode in ("opts", "optsc", "layers") else 1), dtype=torch.uint8,
                        device="cuda") for hb in hbs]
    if mode == "encap":                        # the tunnel parse's outer + tunnel records
        tpar = [engine.parse_tunnel_batch(db, pflags)[:2] for db in dbs]
    if mode == "tunnel":                       # outer records, tunnels, inner records
        outs = [(torch.empty(hb.n * REC_BYTES, dtype=torch.uint8, device="cuda"),
                 torch.empty(hb.n * 16, dtype=torch.uint8, device="cuda"),
                 torch.empty(hb.n * REC_BYTES, dtype=torch.uint8, device="cuda")) for hb in hbs]
    if mode == "fields":                       # the walk once, outside the timed region
        lays = [engine.layers_batch(db) for db in dbs]
        reqs = fields.requests(FIELD_LEG)
        vals = [torch.empty((hb.n, len(FIELD_LEG)), dtype=torch.int64, device="cuda")
                for hb in hbs]
        pres = [torch.empty(hb.n, dtype=torch.int32, device="cuda") for hb in hbs]
    forbid = engine.forbid_list([ip_u32(x) for x in FORBID_IPS])
    dmac, smac = bytes([0xAC, 0xDC, 0xCA, 0x79, 0xCA, 0x86]), bytes([0xAC, 0xDC, 0xCA, 0x79, 0xE5, 0xC6])
    stream = torch.cuda.current_stream()

    def one(k):
        j = k % R
        if mode == "build":
            engine.build_batch(dbs[j], recs[j], 3, built=outs[j], stream=stream)
        elif mode == "opts":
            engine.options_batch(dbs[j], recs[j], opts=outs[j], stream=stream)
        elif mode == "optsc":
            engine.options_batch(dbs[j], recs16[j], opts=outs[j], stream=stream, compact=True)
        elif mode == "layers":
            engine.layers_batch(dbs[j], out=outs[j], stream=stream)
        elif mode == "fields":
            engine.fields_batch(dbs[j], lays[j], reqs, values=vals[j], present=pres[j],
                                stream=stream)
        elif mode == "tunnel":
            o, t, i = outs[j]
            engine.parse_tunnel_batch(dbs[j], pflags, outer=o, tun=t, inner=i, stream=stream)
        elif mode == "encap":
            engine.build_tunnel_batch(dbs[j], tpar[j][0], tpar[j][1], 3, built=outs[j],
                                      stream=stream)
        else:
            engine.forward_batch(dbs[j], dmac, smac, forbid, keep=outs[j], stream=stream,
                                 flags=fwd_flags)

    k, t_w = 0, time.perf_counter()
    while k < args.warmup or time.perf_counter() - t_w < args.min_warmup_s:
        one(k)
        k += 1
        if k % 16 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier(world)
    t0 = time.perf_counter()
    ev0.record(stream)
    for k in range(args.steps):
        one(k)
    ev1.record(stream)
    torch.cuda.synchronize()
    wall = max_over_ranks(time.perf_counter() - t0, world)
    kern_ms = ev0.elapsed_time(ev1) / args.steps
    r = as_records(recs[0].cpu().numpy())
    lens = hbs[0].lens()
    # header bytes the build writes: link + IPv4 header (or the IPv6 header's first 8
    # bytes) + the fixed L4 header
    six = is_ip6(r)
    l4fix = np.where(r["ip_protocol"] == 17, 8, 20)
    fixed = np.where(six, r["l3_off"].astype(np.int64) + 8 + l4fix,
                     r["l4_off"].astype(np.int64) + l4fix)
    floor = None                               # the 128-B line floor of the reads + writes
    fo = hbs[0].offsets[:-1].astype(np.int64) if hbs[0].offsets is not None else \
        np.arange(hbs[0].n, dtype=np.int64) * hbs[0].stride
    if mode == "build":
        alg = int(lens.sum()) + hbs[0].n * REC_BYTES + int(fixed.sum())
    elif mode == "tunnel":                     # every frame byte once + 80 + 16 + 80 B written
        alg = int(lens.sum()) + hbs[0].n * (2 * REC_BYTES + 16)
    elif mode == "encap":                      # records read, the frame read once (sums), the
        tr = as_tunnels(tpar[0][1].cpu().numpy())   # headers up to the tunnel header's end written
        h0 = tr["hdr0"].astype(np.int64)
        thl = np.select([tr["kind"] == 1, tr["kind"] == 2],
                        [8, np.where(h0 & 7, 12, 8)],
                        4 + 4 * ((h0 & 0xc0) != 0) + 4 * ((h0 & 0x20) != 0) + 4 * ((h0 & 0x10) != 0))
        alg = int(lens.sum()) + hbs[0].n * (REC_BYTES + 16) + \
            int((tr["tun_off"].astype(np.int64) + thl).sum())
    elif mode == "layers":                       # header bytes walked + 64 B out per frame
        lo = outs[0].cpu().numpy().view(LAYERS_DTYPE)
        walked = np.minimum(lo["payload_off"].astype(np.int64), lens)
        alg = int(walked.sum()) + hbs[0].n * 64
        floor = line_floor(fo, fo + walked) + hbs[0].n * 64
    elif mode == "fields":                     # layer records + field bytes read, values written
        pm = pres[0].cpu().numpy().view(np.uint32)
        nbytes = [(int(q["bit_off"]) + int(q["bits"]) - 1) // 8 - int(q["bit_off"]) // 8 + 1
                  for q in reqs]
        got = sum(int(((pm >> r) & 1).sum()) * nb for r, nb in enumerate(nbytes))
        alg = hbs[0].n * (64 + 8 * len(reqs) + 4) + got
        # the lines holding the fields read: each present request's bytes at the offset of
        # the nth layer of its protocol (rpkt_gpu_fields_batch's rule)
        lay = lays[0].cpu().numpy().view(LAYERS_DTYPE)
        live = np.arange(16)[None, :] < lay["n"].astype(np.int64)[:, None]
        rows = np.arange(hbs[0].n)
        s0, s1 = [], []
        for r, q in enumerate(reqs):
            hit = (lay["proto"] == q["proto"]) & live
            sel = hit & (np.cumsum(hit, axis=1) == int(q["nth"]) + 1)
            has = sel.any(axis=1) & (((pm >> r) & 1) != 0)
            off = lay["off"][rows, sel.argmax(axis=1)].astype(np.int64)
            b0 = off + int(q["bit_off"]) // 8
            b1 = off + (int(q["bit_off"]) + int(q["bits"]) - 1) // 8 + 1
            s0.append(np.where(has, fo + b0, 0))
            s1.append(np.where(has, fo + b1, 0))
        floor = hbs[0].n * (64 + 8 * len(reqs) + 4) + line_floor(np.concatenate(s0),
                                                                 np.concatenate(s1))
    elif mode in ("opts", "optsc"):            # records + option slices read, 64 B written
        ip_parsed = ((r["status"] == 0) | (r["status"] >= 9)) & ~is_ip6(r)   # Ipv4OptionsIter
        tcp = (r["status"] == 0) & (r["ip_protocol"] == 6)
        l3, l4 = r["l3_off"].astype(np.int64), r["l4_off"].astype(np.int64)
        po = r["payload_off"].astype(np.int64)
        # Ipv6OptionsIter: the extension chain [l3 + 40, l4) of an IPv6 record is walked
        ip6_walked = is_ip6(r) & (l4 >= l3 + 40) & (r["status"] != 14) & (r["status"] != 15)
        slices = np.where(ip_parsed, l4 - l3 - 20, 0) + np.where(tcp, po - l4 - 20, 0) + \
            np.where(ip6_walked, l4 - l3 - 40, 0)
        fixed_io = hbs[0].n * ((REC16_BYTES if mode == "optsc" else REC_BYTES) + 64)
        alg = fixed_io + int(slices.sum())
        floor = fixed_io + line_floor(
            np.concatenate([np.where(ip_parsed, fo + l3 + 20, 0), np.where(tcp, fo + l4 + 20, 0),
                            np.where(ip6_walked, fo + l3 + 40, 0)]),
            np.concatenate([np.where(ip_parsed, fo + l4, 0), np.where(tcp, fo + po, 0),
                            np.where(ip6_walked, fo + l4, 0)]))
    elif mode == "forward":
        kept = outs[0].cpu().numpy().astype(bool)
        # rewritten bytes of a kept frame: 0 .. l4 + 8 (IPv4: 42; IPv6: 62 and up)
        alg = int(lens.sum()) + hbs[0].n + int((r["l4_off"][kept].astype(np.int64) + 8).sum())
    achieved = alg / (kern_ms / 1e3) / 1e9
    traffic, tsrc = pmc_traffic_tx("%s%d" % (mode, cfg), hbs[0].n)   # the bench leg's name
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu and args.tx_cpu_seconds > 0:
        # the leg's CPU restatement beside it: the oracle over the batch's first frames
        # (<= 64 MB), 1 thread, outputs allocated once outside the timed calls
        oracle, build = oracle_for_baseline()
        hs = head_sample(hbs[0], 64 << 20)
        m = hs.n
        kw = dict(offsets=hs.offsets, stride=hs.stride, frame_len=hs.frame_len)
        if mode == "encap":
            kw.update(recs=as_records(tpar[0][0].cpu().numpy())[:m],
                      tun=as_tunnels(tpar[0][1].cpu().numpy())[:m], flags=3)
        elif mode == "tunnel":
            kw.update(flags=pflags)
        elif mode == "fields":
            kw.update(layers=lays[0].cpu().numpy().view(LAYERS_DTYPE)[:m], reqs=reqs)
        elif mode == "forward":
            kw.update(recs=r[:m], flags=fwd_flags, dmac=dmac, smac=smac,
                      forbid=[ip_u32(x) for x in FORBID_IPS])
        elif mode != "layers":
            kw.update(recs=r[:m], flags=3)
        reps, dt = timed_reps(oracle.leg_callable(mode, hs.frames, m, **kw), args.tx_cpu_seconds)
        cpu = {"value": round(m * reps / dt / 1e6, 3), "unit": "Mpps", "cores": 1, "kind": "port",
               "sample": "%d reps x first %d frames (%.0f MB) of the batch, 1 thread"
                         % (reps, m, hs.lens().sum() / 1e6),
               "seconds": round(dt, 2), "build": build}
    return {"mpps": hbs[0].n * world * args.steps / wall / 1e6, "kernel_ms": kern_ms,
            "cpu_baseline": cpu,
            "ms_per_step": wall / args.steps * 1e3, "frames_per_rank": hbs[0].n,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "alg_bytes_per_launch": alg, "traffic": traffic,
                         "traffic_source": tsrc, "line_floor_bytes": floor,
                         "traffic_over_floor": round(traffic / floor, 4)
                         if traffic and floor else None},
            "what": ("build: Udp|Tcp/Ipv4/Ether prepend_header + setters, IPv4 + L4 checksum "
                     "fill" if mode == "build" else
                     "options: Ipv4OptionsIter + TcpOptionsIter walks of a parsed batch"
                     if mode == "opts" else
                     "options from compact 16-B records (rpkt_gpu_options_batch_compact)"
                     if mode == "optsc" else
                     "layers: pktfmt-derived protocol walk (captures mix, fuzzed)"
                     if mode == "layers" else
                     "fields: %d pktfmt getters per frame over the layer walk (captures mix)"
                     % len(FIELD_LEG) if mode == "fields" else
                     "tunnel: outer parse + VXLAN / GTP-U / GRE decode + inner parse, all four "
                     "sums (rpkt_gpu_parse_tunnel_batch)" if mode == "tunnel" else
                     "encap: outer headers + VXLAN / GTP-U / GRE header + IPv4, UDP and GRE "
                     "checksum fill (rpkt_gpu_build_tunnel_batch)" if mode == "encap" else
                     "forward: loopback_rx firewall fused (parse + both sums, 8 forbidden "
                     "sources, swap + ttl-1 + MACs + checksum update)")}


LINE_MAX = 8000           # the driver keeps an 8,000-char tail of stdout: the line fits it
CPU_KEYS = ("value", "unit", "cores", "kind", "sample", "gb_per_s", "all_cores_mpps",
            "all_cores_gb_per_s", "all_cores_threads", "all_cores_scaling", "gpu_parity_on_sample",
            "cpu_model")
FLOW_KEYS = ("flow_reduce_ms", "flow_reduce_ms_min", "flow_reduce_ms_max", "flow_reduce_samples",
             "flow_reduce_via", "flow_reduce_verified", "flow_reduce_error", "flow_pkts_total",
             "flow_pkts_expected")
REDUCE_SAMPLES = 20       # counter reduces timed per config-4 leg (median, min, max reported)


def _r(x, nd=4):
    return round(x, nd) if isinstance(x, float) else x


def leg_summary(v):
    """One extra leg in the stdout line: its kernel time, step time, roofline fraction and
    PMC traffic over algorithmic bytes (the rest of the leg is in the detail file)."""
    if "roofline" in v:
        rf = v["roofline"]
        t, a = rf.get("traffic"), rf.get("alg_bytes_per_launch")
        s = {"kernel_ms": _r(v.get("kernel_ms"), 5), "ms_per_step": _r(v.get("ms_per_step"), 5),
             "frac": rf.get("frac"), "traffic_ratio": round(t / a, 4) if t and a else None}
        if "achieved_all_ranks" in rf:
            s["achieved_all_ranks"] = rf["achieved_all_ranks"]
        for k in ("mpps", "flow_reduce_ms", "flow_reduce_ms_min", "flow_reduce_ms_max",
                  "flow_reduce_via", "flow_reduce_verified"):
            if k in v:
                s[k] = _r(v[k], 3)
        if isinstance(v.get("cpu_baseline"), dict) and "value" in v["cpu_baseline"]:
            s["cpu_mpps"] = v["cpu_baseline"]["value"]        # the oracle, 1 thread
        return s
    if "ns_per_pkt" in v:                                          # config 1 (host CPU)
        return {"ns_per_pkt": v["ns_per_pkt"], "mpps": v["mpps"], "cores": v["cores"]}
    # nested legs (host_inclusive, rx_graph): the rate of every sub-leg, checks kept
    out = {}
    for k, sub in v.items():
        if isinstance(sub, dict):
            out[k] = (round(sub["mpps"], 1) if "mpps" in sub else
                      {kk: (round(vv["mpps"], 1) if isinstance(vv, dict) and "mpps" in vv else vv)
                       for kk, vv in sub.items()})
            if isinstance(sub, dict) and sub.get("records_checked") is False:
                out[k + "_records_checked"] = False
        else:
            out[k] = _r(sub)
    return out


def headline_line(main_res, extra, args, world, engine_build, detail_path):
    """The one JSON line rank 0 prints: the driver's contract keys, the main leg's
    roofline and CPU baseline (top-level scalars), the flow-reduce fields, and per extra
    leg only its times and fractions.  Always < LINE_MAX bytes: when a leg set would not
    fit, the per-leg summaries shrink to the roofline fraction alone."""
    fb = {2: 64, 3: 1500, 7: 8000, 10: 64, 11: 1500}.get(args.config)
    rf = dict(main_res["roofline"])
    rf.pop("traffic_source", None)
    cpu = main_res.get("cpu_baseline")
    line = {
        "metric": METRIC,
        "value": round(main_res["mpps"], 2),
        "unit": "Mpps",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(main_res["ms_per_step"], 4),
        "higher_is_better": True,
        "scaling": main_res["scaling"],
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (seeded generator, rpkt-dpdk loopback_tx frame shapes)",
        "config": {"workload": WORKLOAD[args.config], "frames_per_rank":
                   main_res["frames_per_rank"], "frame_bytes": fb,
                   "layout": main_res["layout"], "checksums": main_res["flags"],
                   "parallelism": "replicas x%d (independent batches, no collective)" % world
                   if args.config != 4 else "shard x%d + RCCL all-reduce" % world,
                   "dist_backend": args.dist_backend if world > 1 else None,
                   "shared_gpu": bool(args.share_gpu) if world > 1 else None},
        "frame_gb_per_s": round(main_res["frame_gb_per_s"], 2),
        "kernel_ms": round(main_res["kernel_ms"], 5),
        "engine_build": engine_build,
        "roofline": rf,
        "cpu_baseline": {k: cpu[k] for k in CPU_KEYS if k in cpu} if cpu else None,
        "detail": detail_path,
    }
    for k in FLOW_KEYS:
        if k in main_res:
            line[k] = _r(main_res[k], 5)
    if "copy_ceiling" in main_res:
        line["copy_ceiling_gb_per_s"] = {k: v.get("gb_per_s") for k, v in
                                         main_res["copy_ceiling"].items() if isinstance(v, dict)}
    # flow-reduce fields of an extra config-4 leg at the top level too (the N-rank check)
    for k in FLOW_KEYS:
        if k not in line and "config4" in extra and k in extra["config4"]:
            line[k] = _r(extra["config4"][k], 5)
    line["extra"] = {k: leg_summary(v) for k, v in extra.items()}
    if len(json.dumps(line)) >= LINE_MAX:
        line["extra"] = {k: (s.get("frac") if "frac" in s else s.get("mpps"))
                         for k, s in line["extra"].items()}
    if len(json.dumps(line)) >= LINE_MAX:
        line["extra"] = {"omitted": "see detail"}
    return line


def write_detail(path, main_res, extra, args, world, engine_build):
    """Every leg's full result (what it measured, layouts, line floors, CPU samples) to a
    side file; the stdout line names it."""
    full = {"metric": METRIC, "n_gpus": world, "argv": sys.argv[1:], "engine_build": engine_build,
            "main": main_res, "extra": extra}
    os.makedirs(os.path.dirname(path) or ".", exist_ok=True)
    with open(path, "w") as fh:
        json.dump(full, fh, indent=1, default=lambda o: _r(float(o)) if hasattr(o, "__float__")
                  else str(o))


# legs run by default at N = 1, and at N > 1 unless --all-legs (the N-rank job stays short:
# the headline, config 4's sharded parse + counter reduce, and the strong-scaling legs)
LEG_DEFAULTS = {"also": ("3,4,5,7,10,11", "4"),
                "tx": ("build2,build3,build11,forward2,forward10,opts5,optsc5,opts11,layers9,"
                       "fields9,tunnel13,encap13", ""),
                "compact": ("2,3", ""), "strong": ("2,3", "2,3"), "opts": ("5", ""),
                "ring": ("2,10", "")}


def resolve_legs(args, world):
    for k, (one, many) in LEG_DEFAULTS.items():
        if getattr(args, k) is None:
            setattr(args, k, one if world == 1 or args.all_legs else many)
    return args


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 200 timed launches: the region's fixed ends (the first launch reaching the GPU, the
    # closing synchronize: about 35 us) are 0.2 us of a 26-us step instead of 0.7 at 50
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", type=int, default=2, choices=[2, 3, 4, 5, 7, 10, 11])
    ap.add_argument("--also", default=None,
                    help="extra configs reported under 'extra' (default 3,4,5,7,10,11; 4 at N>1)")
    ap.add_argument("--frames", type=int, default=0, help="override frames per batch")
    ap.add_argument("--rotate", type=int, default=0, help="distinct batches per rank")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="all-cores CPU leg threads (0 = every usable host thread)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--tx-cpu-seconds", type=float, default=1.5,
                    help="per TX / walk / tunnel leg: the oracle's 1-thread timing beside it "
                         "(0: off)")
    ap.add_argument("--tx", default=None,
                    help="legs beyond the parse reported under 'extra' (default "
                         "build2,build3,forward2,opts5,optsc5,layers9,fields9; none at N>1) (build<cfg>, "
                         "forward<cfg>, opts<cfg>, optsc<cfg> (compact records), layers9, "
                         "fields9)")
    ap.add_argument("--min-warmup-s", type=float, default=0.3,
                    help="extend the W warmup steps to at least this much GPU time")
    ap.add_argument("--reduce-comm", default="auto", choices=["own", "auto", "torch"],
                    help="flow-counter reduce: rpkt_gpu_flow_reduce on torch's RCCL communicator "
                         "(auto, the default), on the library's own, joined with a deadline "
                         "(own), or torch's all_reduce (torch)")
    ap.add_argument("--dist-backend", default="nccl",
                    help="nccl (RCCL over xGMI); gloo only to rehearse N>1 on one GPU")
    ap.add_argument("--share-gpu", action="store_true",
                    help="rehearse N nccl ranks on fewer GPUs (rank r on cuda:r %% ndev; a "
                         "distinct NCCL_HOSTID per rank, RCCL over loopback sockets)")
    ap.add_argument("--no-config1", action="store_true", help="skip the config-1 CPU leg")
    ap.add_argument("--record", default="full", choices=["full", "compact"],
                    help="record size of the main leg (profiling the compact kernel alone)")
    ap.add_argument("--main-opts", action="store_true",
                    help="main leg as the fused parse + option walks (profiling it alone)")
    ap.add_argument("--compact", default=None,
                    help="configs also timed with 16-B compact records (extra.config<N>_compact)")
    ap.add_argument("--host", default="2,3",
                    help="configs also timed host-inclusive at N=1 (pinned H2D frames -> parse "
                         "-> D2H records, rpkt_amd.pipeline): extra.host_inclusive")
    ap.add_argument("--rx-graph", default="16384x64,65536x16",
                    help="receive loops of small config-2 batches, FRAMESxSLOTS, timed eager "
                         "and as a replayed hipGraph at N=1 (rpkt_amd.graphs): extra.rx_graph")
    ap.add_argument("--strong", default=None,
                    help="configs also timed as one batch split over the ranks "
                         "(extra.config<N>_strong)")
    ap.add_argument("--ring", default=None,
                    help="configs also timed as 8 full batches per rpkt_gpu_parse_ring launch "
                         "(default 2,10; none at N>1) "
                         "(extra.config<N>_ring8[_compact])")
    ap.add_argument("--opts", default=None,
                    help="configs also timed as the fused parse + option walks "
                         "(extra.config<N>_opts, extra.config<N>_opts_compact)")
    ap.add_argument("--all-legs", action="store_true",
                    help="at N>1, run every N=1 default leg too (longer job)")
    ap.add_argument("--detail", default=os.path.join(ROOT, "gpurun_out", "bench_detail.json"),
                    help="side file with every leg's full result (the stdout line names it)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # no launcher: start the N ranks here (before any GPU call) and wait for them
        sys.exit(launch_ranks(args.gpus, sys.argv[1:], share=args.share_gpu))
    rank, local, world = dist_env()
    # stdout carries ONE line, the JSON result: the libraries loaded below print to fd 1
    # (RCCL's version banner at communicator creation, gloo's peer list), so fd 1 points at
    # stderr for the whole run and the line is written to the saved stdout at the end
    sys.stdout.flush()
    result_fd = os.dup(1)
    os.dup2(2, 1)
    if args.share_gpu and args.dist_backend == "nccl":
        for k, v in share_gpu_env(rank).items():      # read by RCCL at communicator init
            os.environ.setdefault(k, v)
    if world != args.gpus:
        print("[bench] error: %d rank(s) launched for --gpus %d" % (world, args.gpus),
              file=sys.stderr)
        sys.exit(3)
    ndev = torch.cuda.device_count()                 # counts without initialising HIP
    shared = args.dist_backend == "gloo" or args.share_gpu
    if args.dist_backend == "nccl" and local >= ndev and not args.share_gpu:
        print("[bench] error: rank %d needs cuda:%d but %d GPU(s) are visible (use "
              "--dist-backend gloo to rehearse ranks on one GPU)" % (rank, local, ndev),
              file=sys.stderr)
        sys.exit(3)
    dev = local % ndev if shared else local
    torch.cuda.set_device(dev)
    if world > 1:
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group("gloo")
        if dist.get_world_size() != args.gpus:
            print("[bench] error: world size %d != --gpus %d" % (dist.get_world_size(),
                                                                  args.gpus), file=sys.stderr)
            sys.exit(3)
    resolve_legs(args, world)
    want_cpu = (not args.no_cpu) and world == 1
    if not args.cpu_threads:
        args.cpu_threads = usable_cpus()

    main_res = run_config(args.config, args, rank, world, cpu=want_cpu and not args.main_opts,
                          compact=args.record == "compact", opts=args.main_opts, main=True)
    extra = {}
    for c in [int(x) for x in args.also.split(",") if x.strip()]:
        if c != args.config:
            extra["config%d" % c] = run_config(c, args, rank, world, cpu=want_cpu)
    for leg, mode, cfg in tx_legs(args.tx):
        extra["tx_" + leg] = run_tx(cfg, mode, args, rank, world)
    for c in [int(x) for x in args.compact.split(",") if x.strip()]:
        extra["config%d_compact" % c] = run_config(c, args, rank, world, compact=True)
    for c in [int(x) for x in args.strong.split(",") if x.strip()]:
        extra["config%d_strong" % c] = run_config(c, args, rank, world, strong=True)
    for c in [int(x) for x in args.opts.split(",") if x.strip()]:
        extra["config%d_opts" % c] = run_config(c, args, rank, world, opts=True)
        extra["config%d_opts_compact" % c] = run_config(c, args, rank, world, compact=True,
                                                        opts=True)
    for c in [int(x) for x in args.ring.split(",") if x.strip()]:
        extra["config%d_ring8" % c] = run_ring(c, args, rank, world)
        extra["config%d_ring8_compact" % c] = run_ring(c, args, rank, world, compact=True)
    if world == 1 and args.host.strip():
        extra["host_inclusive"] = run_host(args)
    if world == 1 and args.rx_graph.strip():
        extra["rx_graph"] = run_rx_graph(args)
    if want_cpu and not args.no_config1:
        extra["config1"] = run_config1(args)

    if rank == 0:
        build = engine.lib().rpkt_gpu_build_info().decode()
        detail = os.path.relpath(args.detail, ROOT)
        try:
            write_detail(args.detail, main_res, extra, args, world, build)
        except OSError as e:
            detail = "not written: %s" % e
        line = headline_line(main_res, extra, args, world, build, detail)
        sys.stdout.flush()
        os.write(result_fd, (json.dumps(line) + "\n").encode())
    # a counter sum that is wrong (not merely taken by the fallback path) fails the run
    bad_counters = any(r.get("flow_reduce_verified") is False or
                       r.get("flow_pkts_total", 0) != r.get("flow_pkts_expected", 0)
                       for r in [main_res] + list(extra.values()))
    if world > 1:
        dist.barrier()
        rdist.release_own_comms()
        dist.destroy_process_group()
    if bad_counters:
        print("[bench] error: flow counters wrong after the reduce (see flow_reduce_error)",
              file=sys.stderr)
        sys.exit(4)


if __name__ == "__main__":
    main()
