#!/bin/bash
# layer walk: record entries in registers (A, product) vs per-lane LDS records (B:
# -DRPKT_LAY_LDSREC=1, 51.5 KB per block: 3 blocks per CU instead of 4)
set -o pipefail
OUT=gpurun_out/ab_ldsrec
mkdir -p $OUT
for leg in layers9 layers2 layers5; do
  timeout -k 10 200 python3 -u tools/ab_lib.py rpkt_amd/_build_ldsrec/librpkt_gpu.so --leg $leg --rounds 8 --launches 20 \
    > $OUT/ab_$leg.log 2>&1 || exit 1
done
