#!/bin/bash
# layer walk: the ended record stored after the next frame's window loads are issued
# (same process vs the product, outputs compared)
set -o pipefail
O=gpurun_out/r03_laylate
mkdir -p $O
for leg in layers9 layers2 layers5; do
  timeout -k 10 150 python3 -u tools/ab_lib.py rpkt_amd/_ab/late/librpkt_gpu.so --leg $leg --rounds 7 >> $O/late.log 2>&1 || exit 1
done
