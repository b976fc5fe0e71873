#!/bin/bash
# same-process A/B of the flow counters (histogram + slab reduce) on config 4's events
set -o pipefail
mkdir -p gpurun_out/ab_flow
for b in fu16 fu32 ru16 rs2 rs4; do
  timeout -k 10 300 python3 -u tools/ab_lib.py rpkt_amd/_build_$b/librpkt_gpu.so --leg flow4 --rounds 8 --launches 20 \
    > gpurun_out/ab_flow/ab_flow4_$b.log 2>&1 || exit 1
done
