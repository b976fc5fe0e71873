#!/bin/bash
# layer walk: smaller windows (96 / 80 B) for 5 / 6 waves per SIMD, pool sized to the wave slots
set -o pipefail
mkdir -p gpurun_out/ab_layers_occ
for b in c6 c5 c8a; do
  for leg in layers9 layers2; do
    timeout -k 10 200 python3 -u tools/ab_lib.py rpkt_amd/_build_$b/librpkt_gpu.so --leg $leg --rounds 8 --launches 20 \
      > gpurun_out/ab_layers_occ/ab_${leg}_$b.log 2>&1 || exit 1
  done
done
