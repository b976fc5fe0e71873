#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/spec
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_layers.py tests/test_gpu_fields.py -x -q --timeout 120 --timeout-method thread > gpurun_out/spec/pytest.log 2>&1 && \
for c in 9 2 5; do
timeout -k 10 300 python3 -u tools/ablate_layers.py --config $c --frames 4,1004,2,1,8 --rounds 3 > gpurun_out/spec/ablate_c$c.log 2>&1 || exit 1
done
