#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/wf
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_walk_fields.py tests/test_gpu_layers.py -x -q --timeout 200 --timeout-method thread > gpurun_out/wf/pytest.log 2>&1 && \
timeout -k 10 300 python3 -u bench.py --also "" --compact "" --no-cpu --no-config1 --tx layers9,fields9,walkfields9 > gpurun_out/wf/bench.json 2> gpurun_out/wf/bench.log
