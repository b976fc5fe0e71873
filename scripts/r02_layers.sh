#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_layers.py tests/test_gpu_fields.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r02_pytest_layers.log 2>&1 && \
timeout -k 10 300 python3 -u tools/ablate_layers.py > gpurun_out/r02_ablate_layers.log 2>&1
