#!/bin/bash
# field getters staged per request group: 8 requests in flight (A, 74 VGPRs, 6 waves
# per SIMD) vs 16 (B: _build_fg16, 114 VGPRs) and 4 (B: _build_fg4, 60 VGPRs)
set -o pipefail
OUT=gpurun_out/ab_fgroup
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fields.py -x -q --timeout 120 --timeout-method thread \
    > $OUT/tests.log 2>&1 || exit 1
for b in fg16 fg4; do
  timeout -k 10 200 python3 -u tools/ab_lib.py rpkt_amd/_build_$b/librpkt_gpu.so --leg fields9 --rounds 8 --launches 20 \
    > $OUT/ab_$b.log 2>&1 || exit 1
done
