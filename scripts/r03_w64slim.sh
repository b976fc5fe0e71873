#!/bin/bash
# compact parse of 64-B frames: the 64-B-window compile without the record-stage floor
# on its window area (7 blocks per CU instead of 6); same process, outputs compared
set -o pipefail
O=gpurun_out/r03_w64slim
mkdir -p $O
for r in 1 2; do
  timeout -k 10 150 python3 -u tools/ab_lib.py rpkt_amd/_ab/w64slim/librpkt_gpu.so --leg parsec2 --rounds 9 >> $O/ab.log 2>&1 || exit 1
done
