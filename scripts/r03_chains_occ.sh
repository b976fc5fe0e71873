#!/bin/bash
# chains kernel compiled for 3 / 4 blocks per CU (B; 20 / 114 VGPRs spilled) against 2 (A)
set -o pipefail
O=gpurun_out/r03_chains_occ
mkdir -p $O
for b in 3 4; do
  timeout -k 10 200 python3 -u tools/ab_lib.py rpkt_amd/_ab/ch$b/librpkt_gpu.so --leg chains7 --rounds 5 >> $O/ab.log 2>&1 || exit 1
done
