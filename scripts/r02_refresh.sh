#!/bin/bash
# refresh every profile the bench line cites, then the default bench (1 GPU)
set -o pipefail
mkdir -p gpurun_out
bash scripts/refresh_profiles.sh > gpurun_out/r02_refresh.log 2>&1 && \
timeout -k 10 900 python3 -u bench.py > gpurun_out/r02_bench3.json 2> gpurun_out/r02_bench3.log
