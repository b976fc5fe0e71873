#!/bin/bash
# same-process A/B of the 64-B-window TX compile: whole-frame (product) vs the stream
# kept, and vs occupancy capped at 5 / 4 waves per SIMD by dynamic LDS
set -o pipefail
mkdir -p gpurun_out/whole_r8
for b in whole0 pad5 pad4 w64off; do
  for leg in forward2 build2; do
    timeout -k 10 200 python3 -u tools/ab_lib.py rpkt_amd/_build_$b/librpkt_gpu.so --leg $leg --rounds 8 --launches 24 \
      > gpurun_out/whole_r8/ab_${leg}_$b.log 2>&1 || exit 1
  done
done
