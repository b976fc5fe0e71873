#!/bin/bash
# where the fused walk's time goes: same-process A/B of the fused parse + option walks
# against builds without the walks / without the window refill, and the parse alone
set -o pipefail
O=gpurun_out/r03_optabl
mkdir -p $O
for b in nowalk norefill unpaired; do
  timeout -k 10 300 python3 -u tools/ab_lib.py rpkt_amd/_ab/$b/librpkt_gpu.so --leg popts5 --rounds 7 > $O/ab_$b.log 2>&1 || exit 1
done
timeout -k 10 300 python3 -u tools/ab_lib.py rpkt_amd/_ab/nowalk/librpkt_gpu.so --leg parse5 --rounds 7 > $O/ab_parse5.log 2>&1
