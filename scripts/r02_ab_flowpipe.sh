#!/bin/bash
# flow histogram with the next events loaded before the atomics and 1024 threads per
# block (A) vs the same without the prefetch (B: _build_nopipe) and the previous product
# (B: _build_ft512, 512 threads, no prefetch); 8M and 1M IMIX events; flow GPU tests
set -o pipefail
OUT=gpurun_out/ab_flowpipe
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_dist.py -x -q -k "flow or dist" --timeout 120 --timeout-method thread \
    > $OUT/tests.log 2>&1 || exit 1
for b in nopipe ft512; do
  timeout -k 10 200 python3 -u tools/ab_lib.py rpkt_amd/_build_$b/librpkt_gpu.so --leg flow4 --rounds 8 --launches 20 \
    > $OUT/ab_${b}_8m.log 2>&1 || exit 1
  timeout -k 10 200 python3 -u tools/ab_lib.py rpkt_amd/_build_$b/librpkt_gpu.so --leg flow4 --n 1048576 --rounds 8 --launches 20 \
    > $OUT/ab_${b}_1m.log 2>&1 || exit 1
done
