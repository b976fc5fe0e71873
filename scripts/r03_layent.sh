#!/bin/bash
# layer walk: the record's per-layer entries in the slot (LDS) instead of 12 registers,
# 80- / 64-B windows (same LDS per block); same process vs the product, outputs compared
set -o pipefail
O=gpurun_out/r03_layent
mkdir -p $O
for b in le5 le4; do
  for leg in layers9 layers2 layers5; do
    timeout -k 10 150 python3 -u tools/ab_lib.py rpkt_amd/_ab/$b/librpkt_gpu.so --leg $leg --rounds 7 >> $O/$b.log 2>&1 || exit 1
  done
done
