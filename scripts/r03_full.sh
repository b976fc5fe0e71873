#!/bin/bash
# Everything the round's numbers come from, in one GPU call: the GPU test suite,
# smoke(), every profile (refresh_profiles.sh) and the default bench line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
O=$R/gpurun_out/r03_full
mkdir -p "$O"
cd "$R" && \
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 && \
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 && \
bash scripts/refresh_profiles.sh && \
timeout -k 10 900 python3 -u bench.py > "$O/bench.json" 2> "$O/bench.log"
