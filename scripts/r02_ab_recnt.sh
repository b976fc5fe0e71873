#!/bin/bash
# layer walk: record stores non-temporal (A, product) vs default policy (B: _build_recdef)
set -o pipefail
OUT=gpurun_out/ab_recnt
mkdir -p $OUT
for leg in layers9 layers2 layers5; do
  timeout -k 10 200 python3 -u tools/ab_lib.py rpkt_amd/_build_recdef/librpkt_gpu.so --leg $leg --rounds 8 --launches 20 \
    > $OUT/ab_$leg.log 2>&1 || exit 1
done
