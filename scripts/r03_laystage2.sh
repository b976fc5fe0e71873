#!/bin/bash
# layer walk: staged 64-B record stores and cooperative window fills when many walks
# end together (same process vs the product build, outputs compared)
set -o pipefail
O=gpurun_out/r03_laystage2
mkdir -p $O
for b in ls16 lsc16 lsc8 lsc16_4rt; do
  for leg in layers9 layers2 layers5; do
    timeout -k 10 150 python3 -u tools/ab_lib.py rpkt_amd/_ab/$b/librpkt_gpu.so --leg $leg --rounds 7 >> $O/$b.log 2>&1 || exit 1
  done
done
