#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/ablate.py --configs 2 --rotate 8 --variants 21,45,0 --rounds 10 --launches 20 > gpurun_out/r02_ablate_c2_v21.log 2>&1
