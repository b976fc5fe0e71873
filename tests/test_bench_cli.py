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
    ap_default = [a for a in open(bench.__file__).read().split("\n") if '"--tx", default=' in a][0]
    bench.tx_legs(ap_default.split('default="')[1].split('"')[0])


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
