#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/unroll
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/unroll/pytest.log 2>&1 && \
timeout -k 10 300 python3 -u tools/ablate_fwd.py > gpurun_out/unroll/ablate_fwd.log 2>&1 && \
timeout -k 10 300 python3 -u tools/ablate.py --configs 3,4,5 --variants 0,44 --rounds 3 --launches 10 > gpurun_out/unroll/ablate_parse.log 2>&1 && \
timeout -k 10 300 python3 -u bench.py --also "" --compact "" --no-cpu --no-config1 > gpurun_out/unroll/bench.json 2> gpurun_out/unroll/bench.log
