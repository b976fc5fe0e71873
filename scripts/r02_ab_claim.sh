#!/bin/bash
# layer walk: the block pool handed out in 64-frame tiles per wave (A) vs one LDS atomic
# per step with finishers (B: _build_noclaim); layer/field GPU tests first
set -o pipefail
OUT=gpurun_out/ab_claim
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_layers.py tests/test_gpu_fuzz_layouts.py -x -q --timeout 120 --timeout-method thread \
    > $OUT/tests.log 2>&1 || exit 1
for leg in layers9 layers2 layers5; do
  timeout -k 10 200 python3 -u tools/ab_lib.py rpkt_amd/_build_noclaim/librpkt_gpu.so --leg $leg --rounds 8 --launches 20 \
    > $OUT/ab_$leg.log 2>&1 || exit 1
done
