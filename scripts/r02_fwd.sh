#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/fwd
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_tx.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fwd/pytest.log 2>&1 && \
timeout -k 10 300 python3 -u tools/ablate_fwd.py > gpurun_out/fwd/ablate.log 2>&1 && \
timeout -k 10 300 python3 -u tools/ablate.py --configs 4,3 --variants 0 --rounds 3 --launches 10 > gpurun_out/fwd/ablate_parse.log 2>&1 && \
timeout -k 10 300 python3 -u bench.py --also "" --compact "" --no-cpu --tx build2,forward2 > gpurun_out/fwd/bench.json 2> gpurun_out/fwd/bench.log && \
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_layers.py -x -q --timeout 120 --timeout-method thread > gpurun_out/fwd/pytest_layers.log 2>&1 && \
for c in 9 5; do
timeout -k 10 300 python3 -u tools/ablate_layers.py --config $c --frames 4,104,102,108 --rounds 3 > gpurun_out/fwd/ablate_layers_c$c.log 2>&1 || exit 1
done
