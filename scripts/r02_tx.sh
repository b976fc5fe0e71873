#!/bin/bash
# TX unit changed: its GPU tests, the walks + build3 profiles (traffic_tx.json), and
# the TX legs of the bench on the same box
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
mkdir -p gpurun_out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_tx.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/r02_tx_tests.log 2>&1 && \
bash "$R/scripts/profile.sh" walks 2 --tx layers9,opts5,forward2,build2,fields9 && \
bash "$R/scripts/profile.sh" build3 2 --tx build3 && \
timeout -k 10 300 python3 -u bench.py --no-cpu --no-config1 --also "" --compact "" --tx build2,forward2 \
    > gpurun_out/r02_tx_bench.json 2> gpurun_out/r02_tx_bench.log
