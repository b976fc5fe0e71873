#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for c in 2 3 5 9; do
timeout -k 10 300 python3 -u tools/ablate_layers.py --config $c --frames 1,2,4,404 --rounds 3 > gpurun_out/r02_ablate_layers_c$c.log 2>&1 || exit 1
done
