#!/bin/bash
# after a refresh that stopped at optsc5: that profile, then the default bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
bash "$R/scripts/profile.sh" optsc5 2 --tx optsc5 > gpurun_out/r02_refresh_optsc5.log 2>&1 && \
timeout -k 10 900 python3 -u bench.py > gpurun_out/r02_bench3.json 2> gpurun_out/r02_bench3.log
