#!/bin/bash
# part 2 (configs 5, 7, 3 compact), then the GPU suite, smoke and (WITH_BENCH=1) the
# default bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p gpurun_out
bash "$R/scripts/profile.sh" c5 5 && bash "$R/scripts/profile.sh" c7 7 && \
bash "$R/scripts/profile.sh" c3_compact 3 --record compact && \
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02_pytest_gpu.log 2>&1 && \
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_smoke.log 2>&1 || exit 1
if [ -n "${WITH_BENCH:-}" ]; then
    timeout -k 10 900 python3 -u bench.py > gpurun_out/r02_bench_final3.json 2> gpurun_out/r02_bench_final3.log
fi
