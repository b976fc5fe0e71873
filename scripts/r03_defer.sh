#!/bin/bash
# deferred-getter paired walk: same-process A/B against the paired walk with per-step
# getters and the unpaired walk, fused and standalone
set -o pipefail
O=gpurun_out/r03_defer
mkdir -p $O
for b in nodefer unpaired; do
  for leg in popts5 poptsc5 opts5 optsc5; do
    timeout -k 10 300 python3 -u tools/ab_lib.py rpkt_amd/_ab/$b/librpkt_gpu.so --leg $leg --rounds 7 >> $O/ab_$b.log 2>&1 || exit 1
  done
done
