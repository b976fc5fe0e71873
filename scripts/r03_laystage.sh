#!/bin/bash
# layer walk: records stored through the slots (64-B writes), same process vs the product
set -o pipefail
O=gpurun_out/r03_laystage
mkdir -p $O
for b in laystage laystage4rt laystage6rt; do
  for leg in layers9 layers2; do
    timeout -k 10 150 python3 -u tools/ab_lib.py rpkt_amd/_ab/$b/librpkt_gpu.so --leg $leg --rounds 7 >> $O/$b.log 2>&1 || exit 1
  done
done
