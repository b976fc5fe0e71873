#!/bin/bash
# flow counters at 1M events (config 4 at 8 ranks): fewer, fuller slabs
set -o pipefail
OUT=gpurun_out/ab_flow_small
mkdir -p $OUT
for m in 4096 8192 16384; do
  timeout -k 10 200 python3 -u tools/ab_lib.py rpkt_amd/_build_fm$m/librpkt_gpu.so --leg flow4 --n 1048576 --rounds 8 --launches 40 \
    > $OUT/ab_flow4_1M_fm$m.log 2>&1 || exit 1
done
timeout -k 10 200 python3 -u tools/ab_lib.py rpkt_amd/_build_fm4096/librpkt_gpu.so --leg flow4 --n 2097152 --rounds 8 --launches 40 \
    > $OUT/ab_flow4_2M_fm4096.log 2>&1 || exit 1
