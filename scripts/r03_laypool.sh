#!/bin/bash
# layer walk: window chunks (4/5/6/8 x 16 B) with run-time block pools (one round of
# resident blocks), same process against the product build, outputs compared
set -o pipefail
O=gpurun_out/r03_laypool
mkdir -p $O
for b in lay8rt lay6rt lay5rt lay4rt; do
  for leg in layers9 layers2; do
    timeout -k 10 150 python3 -u tools/ab_lib.py rpkt_amd/_ab/$b/librpkt_gpu.so --leg $leg --rounds 7 >> $O/$b.log 2>&1 || exit 1
  done
done
