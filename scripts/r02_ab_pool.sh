#!/bin/bash
# layer walk with runtime-sized block pools (A: one resident pass of blocks) vs the
# fixed 1024-frame pools (B1: _build_base), and per-lane LDS records with runtime pools
# (B2: _build_ldsrec, 3 blocks per CU); layer GPU tests on A first
set -o pipefail
OUT=gpurun_out/ab_pool
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_layers.py tests/test_gpu_fields.py -x -q --timeout 120 --timeout-method thread \
    > $OUT/tests.log 2>&1 || exit 1
for leg in layers9 layers2 layers5; do
  timeout -k 10 200 python3 -u tools/ab_lib.py rpkt_amd/_build_base/librpkt_gpu.so --leg $leg --rounds 8 --launches 20 \
    > $OUT/ab_base_$leg.log 2>&1 || exit 1
  timeout -k 10 200 python3 -u tools/ab_lib.py rpkt_amd/_build_ldsrec/librpkt_gpu.so --leg $leg --rounds 8 --launches 20 \
    > $OUT/ab_ldsrec_$leg.log 2>&1 || exit 1
done
