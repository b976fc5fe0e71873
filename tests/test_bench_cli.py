"""bench.py's launcher contract on CPU (nothing here reaches a GPU call): a world that
does not match --gpus is refused before any device work, and the usable-thread count
the all-cores CPU leg uses is sane."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_refuses_mismatched_world():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--no-cpu"], capture_output=True, text=True, timeout=300, env=env,
                       cwd=ROOT)
    assert r.returncode == 3 and "--gpus 2" in r.stderr, r.stderr[-2000:]


def test_usable_cpus_within_affinity():
    sys.path.insert(0, ROOT)
    import bench
    n = bench.usable_cpus()
    assert 1 <= n <= len(os.sched_getaffinity(0)) <= (os.cpu_count() or n)


def test_tx_leg_names():
    """Every default --tx leg parses to a known mode and config (optsc before opts)."""
    sys.path.insert(0, ROOT)
    import bench
    legs = bench.tx_legs("build2,build3,forward2,opts5,optsc5,layers9,fields9")
    assert [(m, c) for _, m, c in legs] == [("build", 2), ("build", 3), ("forward", 2), ("opts", 5),
                                           ("optsc", 5), ("layers", 9), ("fields", 9)]
    with pytest.raises(SystemExit):
        bench.tx_legs("nope2")
    with pytest.raises(SystemExit):
        bench.tx_legs("opts")
    for one, many in [bench.LEG_DEFAULTS["tx"]]:
        bench.tx_legs(one)
        bench.tx_legs(many)


def test_line_floor_matches_brute_force():
    """bench.line_floor (the 128-B line floor of the walk legs' roofline): the bytes of
    the distinct lines any range touches, against a set of line indices."""
    import numpy as np
    sys.path.insert(0, ROOT)
    import bench
    rng = np.random.default_rng(5)
    for _ in range(50):
        n = int(rng.integers(0, 200))
        s = rng.integers(0, 20000, n)
        e = s + rng.integers(-5, 400, n)              # empty and negative ranges included
        lines = set()
        for a, b in zip(s.tolist(), e.tolist()):
            if b > a:
                lines.update(range(a // 128, (b - 1) // 128 + 1))
        assert bench.line_floor(s, e) == 128 * len(lines)
    assert bench.line_floor([], []) == 0
    assert bench.line_floor([127], [129]) == 256 and bench.line_floor([128], [256]) == 128


def _r04_legs():
    """main_res / extra rebuilt from round 4's real 20-KB line (every leg populated)."""
    import json
    with open(os.path.join(ROOT, "profiles", "r04_bench_final.json")) as fh:
        L = json.load(fh)
    main = {"mpps": L["value"], "ms_per_step": L["ms_per_step"], "scaling": L["scaling"],
            "frames_per_rank": L["config"]["frames_per_rank"], "layout": L["config"]["layout"],
            "flags": L["config"]["checksums"], "frame_gb_per_s": L["frame_gb_per_s"],
            "kernel_ms": L["kernel_ms"], "roofline": L["roofline"],
            "cpu_baseline": L["cpu_baseline"], "copy_ceiling": L["copy_ceiling"]}
    return main, dict(L["extra"])


class _Args:
    config, steps, warmup, dist_backend, share_gpu = 2, 20, 5, "nccl", False


def test_headline_line_fits_the_driver_tail():
    """The stdout line built from a fully populated leg set (round 4's, whose 20-KB line
    the driver could not parse, plus 20 more synthetic legs) stays under 8,000 bytes and
    keeps the contract keys, the roofline and the CPU baseline's all-cores scalars."""
    import copy
    import json
    sys.path.insert(0, ROOT)
    import bench
    main, extra = _r04_legs()
    line = bench.headline_line(main, extra, _Args, 1, "x" * 400, "gpurun_out/bench_detail.json")
    s = json.dumps(line)
    assert len(s) < 8000, len(s)
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "config", "roofline",
              "cpu_baseline", "detail"):
        assert k in line, k
    assert line["roofline"]["frac"] == main["roofline"]["frac"]
    for k in ("value", "cores", "kind", "sample", "all_cores_mpps", "all_cores_threads"):
        assert k in line["cpu_baseline"], k
    assert set(line["extra"]) == set(extra)
    assert line["extra"]["config3"]["frac"] == extra["config3"]["roofline"]["frac"]
    assert "what" not in s
    assert line["extra"]["config4"]["flow_reduce_via"] == extra["config4"]["flow_reduce_via"]
    # twice the legs still fits (summaries shrink to the fraction alone)
    more = dict(extra)
    for k, v in extra.items():
        more[k + "_again"] = copy.deepcopy(v)
    line2 = bench.headline_line(main, more, _Args, 8, "x" * 400, "gpurun_out/bench_detail.json")
    assert len(json.dumps(line2)) < 8000
    assert line2["n_gpus"] == 8


def test_n_rank_default_leg_set():
    """At N > 1 the default job is the headline, config 4 (shards + counter reduce) and the
    strong legs; --all-legs restores the N = 1 set; explicit flags win."""
    import argparse
    sys.path.insert(0, ROOT)
    import bench

    def ns(**kw):
        d = {k: None for k in bench.LEG_DEFAULTS}
        d.update(all_legs=False)
        d.update(kw)
        return argparse.Namespace(**d)
    a = bench.resolve_legs(ns(), 8)
    assert (a.also, a.tx, a.compact, a.strong, a.opts, a.ring) == ("4", "", "", "2,3", "", "")
    one = bench.resolve_legs(ns(), 1)
    assert one.tx.startswith("build2") and "4" in one.also.split(",")
    allg = bench.resolve_legs(ns(all_legs=True), 8)
    assert allg.tx == one.tx and allg.also == one.also
    assert bench.resolve_legs(ns(tx="layers9"), 8).tx == "layers9"


@pytest.mark.parametrize("threads", [1, 3])
def test_cpu_baseline_timed_call_allocates_nothing(threads):
    """The CPU baseline's timed body (bench.cpu_parse_callable) writes into a record
    buffer made once: after the untimed first call, a call allocates nothing the size of
    the records (tracemalloc sees numpy's buffers), and the records equal the oracle's."""
    import tracemalloc
    sys.path.insert(0, ROOT)
    import bench
    from oracle import oracle
    from rpkt_amd import gen
    hb = gen.make_batch(2, 4096)
    fn = bench.cpu_parse_callable(oracle, hb, gen.FLAGS[2], threads)
    fn()                                               # the untimed first call (first touch)
    rec_bytes = fn.out.nbytes
    tracemalloc.start()
    try:
        base = tracemalloc.get_traced_memory()[0]
        tracemalloc.reset_peak()
        for _ in range(5):
            fn()
        cur, peak = tracemalloc.get_traced_memory()
    finally:
        tracemalloc.stop()
    # (a few KiB of interpreter objects may come and go; a record-sized buffer per call
    # would be 320 KiB here)
    assert peak - base < rec_bytes // 20, (peak - base, rec_bytes)
    assert abs(cur - base) < rec_bytes // 20, (cur, base)
    want = oracle.parse_batch(hb.frames, hb.n, flags=gen.FLAGS[2], stride=hb.stride,
                              frame_len=hb.frame_len)
    assert fn.out.tobytes() == want.tobytes()


def test_packet_l4_all_cores_agrees():
    """Config 1's all-cores loop: every thread's passes find no failed assert, and it
    counts failures like the 1-thread loop on a corrupted frame."""
    sys.path.insert(0, ROOT)
    import numpy as np
    from oracle import oracle
    from rpkt_amd import gen
    hb = gen.make_batch(1)
    r = oracle.parse_batch(hb.frames, hb.n, flags=3, stride=hb.stride)
    keys = ("ip_src", "ip_dst", "ip_checksum", "ip_ident", "src_port", "dst_port",
            "l4_word6", "l4_checksum")
    want = tuple(int(r[k][0]) for k in keys)
    flen = hb.frame_len or hb.stride
    assert oracle.packet_l4_loop_mt(hb.frames, hb.n, hb.stride, flen, 3, want, 4) == 0
    f = np.array(hb.frames, copy=True)
    f[hb.stride * 7 + 40] ^= 0xff                      # frame 7: another source port
    one = oracle.packet_l4_loop(f, hb.n, hb.stride, flen, 2, want)
    assert one == 2
    assert oracle.packet_l4_loop_mt(f, hb.n, hb.stride, flen, 2, want, 4) == 4 * one


@pytest.mark.parametrize("mode,cfg", [("build", 3), ("forward", 2), ("opts", 5), ("layers", 9),
                                      ("fields", 9), ("tunnel", 13), ("encap", 13)])
def test_tx_leg_cpu_callable(mode, cfg):
    """The per-leg CPU timing's body (oracle.leg_callable): after the untimed first call a
    call allocates nothing (tracemalloc), and its outputs are the oracle's own (the in-place
    legs rebuild their private copy identically on every call)."""
    import tracemalloc
    sys.path.insert(0, ROOT)
    import numpy as np
    import bench
    from oracle import oracle
    from rpkt_amd import fields, gen
    hb = gen.make_mix(600, seed=9) if cfg == 9 else gen.make_batch(cfg, 600)
    kw = dict(offsets=hb.offsets, stride=hb.stride, frame_len=hb.frame_len)
    r = oracle.parse_batch(hb.frames, hb.n, flags=gen.FLAGS.get(cfg, 3) | 3, **kw)
    extra = {}
    if mode in ("build", "opts"):
        extra = dict(recs=r, flags=3)
    elif mode == "forward":
        extra = dict(recs=r, flags=0, dmac=b"\xaa" * 6, smac=b"\xbb" * 6, forbid=[1, 2, 3])
    elif mode == "fields":
        extra = dict(layers=oracle.layers_batch(hb.frames, hb.n, **kw),
                     reqs=fields.requests(bench.FIELD_LEG))
    elif mode == "tunnel":
        extra = dict(flags=3)
    elif mode == "encap":
        o, t, _ = oracle.tunnel_batch(hb.frames, hb.n, 3, **kw)
        extra = dict(recs=o, tun=t, flags=3)
    fn = oracle.leg_callable(mode, hb.frames, hb.n, **kw, **extra)
    fn()
    tracemalloc.start()
    try:
        base = tracemalloc.get_traced_memory()[0]
        tracemalloc.reset_peak()
        for _ in range(3):
            fn()
        cur, peak = tracemalloc.get_traced_memory()
    finally:
        tracemalloc.stop()
    assert peak - base < 16384 and abs(cur - base) < 16384, (peak - base, cur - base)
    got = fn.arrays
    if mode == "build":                       # the closure's private copy, built in place
        out, _ = oracle.build_batch(hb.frames, hb.n, r, 3, **kw)
        assert got[2].tobytes() == out.tobytes()
    elif mode == "tunnel":
        want = oracle.tunnel_batch(hb.frames, hb.n, 3, **kw)
        assert all(g.tobytes() == w.tobytes() for g, w in zip(got[2:], want))
    elif mode == "layers":
        assert got[2].tobytes() == oracle.layers_batch(hb.frames, hb.n, **kw).tobytes()
