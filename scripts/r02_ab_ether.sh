#!/bin/bash
# layer walk: the first (Ethernet) step taken with the frame (A) vs in the loop (B)
set -o pipefail
OUT=gpurun_out/ab_ether
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_layers.py tests/test_gpu_fuzz_layouts.py tests/test_gpu_fields.py -x -q --timeout 120 --timeout-method thread \
    > $OUT/tests.log 2>&1 || exit 1
for leg in layers9 layers2 layers5; do
  timeout -k 10 200 python3 -u tools/ab_lib.py rpkt_amd/_build_eth0/librpkt_gpu.so --leg $leg --rounds 8 --launches 20 \
    > $OUT/ab_$leg.log 2>&1 || exit 1
done
