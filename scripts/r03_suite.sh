#!/bin/bash
# full GPU suite + smoke + the default bench line on the current build
set -o pipefail
O=gpurun_out/r03_suite
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 && \
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && \
timeout -k 10 900 python3 -u bench.py > $O/bench.json 2> $O/bench.log
