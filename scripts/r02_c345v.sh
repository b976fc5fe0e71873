#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 -u tools/ablate.py --configs 3,4,5 --variants 0,21 --rounds 3 --launches 10 > gpurun_out/r02_ablate_c345_v21.log 2>&1
