#!/bin/bash
# round 3 start: GPU suite + smoke + default bench line on the round-2 build
set -o pipefail
mkdir -p gpurun_out/r03_start
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03_start/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r03_start/smoke.log 2>&1 && \
timeout -k 10 600 python3 -u bench.py > gpurun_out/r03_start/bench.json 2> gpurun_out/r03_start/bench.log
