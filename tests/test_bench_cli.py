"""bench.py's launcher contract on CPU (nothing here reaches a GPU call): a world that
does not match --gpus is refused before any device work, and the usable-thread count
the all-cores CPU leg uses is sane."""
import os
import subprocess
import sys

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
