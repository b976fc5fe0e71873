#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -k "short_strided or baseline_configs or compact" -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_pytest_w64.log 2>&1 && \
timeout -k 10 200 python3 -u tools/ablate.py --configs 2 --rotate 8 --variants 0,30,1,31,3,33,14 --rounds 5 --launches 20 > gpurun_out/r02_ablate_w64.log 2>&1
