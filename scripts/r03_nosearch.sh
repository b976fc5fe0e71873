#!/bin/bash
# timing ablation: the L4 stream's owner search replaced by a one-range step (B, wrong
# sums) against the product (A); configs 4 and 5 (short ranges, frequent jumps), config 3
set -o pipefail
O=gpurun_out/r03_nosearch
mkdir -p $O
for leg in parse4 parse5 parse3; do
  timeout -k 10 150 python3 -u tools/ab_lib.py rpkt_amd/_ab/nosearch/librpkt_gpu.so --leg $leg --rounds 5 >> $O/ab.log 2>&1 || exit 1
done
