#!/bin/bash
# layer walk: entries stored directly vs inserted into registers (same process, outputs compared)
set -o pipefail
O=gpurun_out/r03_lay
mkdir -p $O
for leg in layers9 layers2 layers5; do
  timeout -k 10 300 python3 -u tools/ab_lib.py rpkt_amd/_ab/laydirect/librpkt_gpu.so --leg $leg --rounds 7 >> $O/ab_direct.log 2>&1 || exit 1
done
