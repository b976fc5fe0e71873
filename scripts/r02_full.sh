#!/bin/bash
# the whole GPU suite, smoke, every profile, and the default bench, on the current build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02_pytest_gpu.log 2>&1 && \
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_smoke.log 2>&1 && \
bash scripts/refresh_profiles.sh > gpurun_out/r02_refresh.log 2>&1 && \
timeout -k 10 900 python3 -u bench.py > gpurun_out/r02_bench3.json 2> gpurun_out/r02_bench3.log
