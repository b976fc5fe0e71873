"""Run bench.py against another build of librpkt_gpu.so (development tool, GPU box):
for PMC profiles of an ablation build, whose kernels carry the product's names.
Usage: python tools/bench_with_lib.py <lib.so> [bench.py args ...]"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from rpkt_amd import engine  # noqa: E402

engine.GPU_LIB = os.path.abspath(sys.argv[1])
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[2:]
runpy.run_path(sys.argv[0], run_name="__main__")
