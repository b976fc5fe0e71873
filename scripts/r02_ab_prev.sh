#!/bin/bash
# in-tree build (A) vs the last commit's (rpkt_amd/_build_prev, B): TX tests + legs
set -o pipefail
OUT=gpurun_out/ab_prev
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_tx.py tests/test_gpu_layers.py tests/test_gpu_fuzz_layouts.py -x -q --timeout 120 --timeout-method thread \
    > $OUT/tests.log 2>&1 || exit 1
for leg in ${LEGS:-forward2 build2}; do
  timeout -k 10 200 python3 -u tools/ab_lib.py rpkt_amd/_build_prev/librpkt_gpu.so --leg $leg --rounds 8 --launches 20 \
    > $OUT/ab_$leg.log 2>&1 || exit 1
done
