#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for R in 8 16 4; do
  timeout -k 10 200 python3 -u tools/ablate.py --configs 2 --rotate $R --variants 0,1,3,8,10,11,12,13,14,15 --rounds 5 --launches 20 > gpurun_out/r02_ablate_c2_R$R.log 2>&1 || exit 1
done
