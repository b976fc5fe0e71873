#!/bin/bash
# where the fused walk's time goes: same-process A/B of the fused parse + option walks
# against builds without the walks / without the window refill / the unpaired walk /
# rules in registers, and the parse alone; then the host-inclusive pipeline sweep
set -o pipefail
O=gpurun_out/r03_optabl
mkdir -p $O
for b in nowalk norefill unpaired rulealu; do
  timeout -k 10 300 python3 -u tools/ab_lib.py rpkt_amd/_ab/$b/librpkt_gpu.so --leg popts5 --rounds 7 > $O/ab_$b.log 2>&1 || exit 1
done
timeout -k 10 300 python3 -u tools/ab_lib.py rpkt_amd/_ab/rulealu/librpkt_gpu.so --leg optsc5 --rounds 7 > $O/ab_rulealu_optsc5.log 2>&1 && \
timeout -k 10 300 python3 -u tools/ab_lib.py rpkt_amd/_ab/nowalk/librpkt_gpu.so --leg parse5 --rounds 7 > $O/ab_parse5.log 2>&1 && \
timeout -k 10 400 python3 -u tools/host_rate.py --configs 2,3 --slots 2,3,4 --groups 1,2,4 > $O/host_rate.log 2>&1
