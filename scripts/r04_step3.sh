#!/bin/bash
# Launch stamps of the config-2 parse at 4 / 2 / 1 waves per block, then the layer
# walk's FETCH/WRITE passes for the in-tree build and the half-refill build
set -o pipefail
O=gpurun_out/r04_step3
mkdir -p $O
timeout -k 10 300 python3 -u tools/launch_stamps.py > $O/stamps.jsonl 2> $O/stamps.log && \
LEGS="" bash scripts/r04_lay.sh
