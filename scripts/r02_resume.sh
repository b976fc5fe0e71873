#!/bin/bash
# re-entry check on the restored tree: GPU suite, smoke, default bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02_pytest_gpu.log 2>&1 && \
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_smoke.log 2>&1 && \
timeout -k 10 900 python3 -u bench.py > gpurun_out/r02_bench_resume.json 2> gpurun_out/r02_bench_resume.log
