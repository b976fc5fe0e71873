#!/bin/bash
# layer walk ablations: refill, record stores, per-frame overhead (ablate lib variants)
set -o pipefail
O=gpurun_out/r03_layabl
mkdir -p $O
timeout -k 10 200 python3 -u tools/ablate_layers.py --frames 104,201,202,203,204,205,206,207 --rounds 7 > $O/c9.log 2>&1 &&
timeout -k 10 200 python3 -u tools/ablate_layers.py --config 2 --frames 104,201,202,203,204,205,206,207 --rounds 7 > $O/c2.log 2>&1
