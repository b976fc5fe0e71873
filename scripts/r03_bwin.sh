#!/bin/bash
# build_kernel window loads non-temporal (B: -DRPKT_BUILD_WIN_AUX=2) against default (A),
# with the records already read non-temporally
set -o pipefail
O=gpurun_out/r03_bwin
mkdir -p $O
for leg in build2 build3; do
  timeout -k 10 200 python3 -u tools/ab_lib.py rpkt_amd/_ab/bwin2/librpkt_gpu.so --leg $leg --rounds 7 >> $O/ab.log 2>&1 || exit 1
done
