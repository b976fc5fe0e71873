#!/bin/bash
# write-back store policy: default (A) vs nt (aux 2) / aux 3
set -o pipefail
OUT=gpurun_out/ab_wb
mkdir -p $OUT
for b in wbnt wbsc; do
  for leg in forward2 build2 build3; do
    timeout -k 10 200 python3 -u tools/ab_lib.py rpkt_amd/_build_$b/librpkt_gpu.so --leg $leg --rounds 8 --launches 20 \
      > $OUT/ab_${leg}_$b.log 2>&1 || exit 1
  done
done
