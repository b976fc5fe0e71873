#!/bin/bash
# flow histogram: 512 threads per block (A, product) vs 1024 / 256 (B builds), 8M and
# 1M IMIX events, same process, identical counters checked by ab_lib
set -o pipefail
OUT=gpurun_out/ab_flowthreads
mkdir -p $OUT
for b in ft1024 ft256; do
  timeout -k 10 200 python3 -u tools/ab_lib.py rpkt_amd/_build_$b/librpkt_gpu.so --leg flow4 --rounds 8 --launches 20 \
    > $OUT/ab_${b}_8m.log 2>&1 || exit 1
  timeout -k 10 200 python3 -u tools/ab_lib.py rpkt_amd/_build_$b/librpkt_gpu.so --leg flow4 --n 1048576 --rounds 8 --launches 20 \
    > $OUT/ab_${b}_1m.log 2>&1 || exit 1
done
