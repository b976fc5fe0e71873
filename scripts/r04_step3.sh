#!/bin/bash
# Launch stamps of the config-2 parse at 4 / 2 / 1 waves per block, then the layer
# walk's FETCH/WRITE passes for the in-tree build and the half-refill build, then the
# walk/TX profiles with the read-request-size pass
set -o pipefail
O=gpurun_out/r04_step3
mkdir -p $O
timeout -k 10 300 python3 -u tools/launch_stamps.py > $O/stamps.jsonl 2> $O/stamps.log && \
LEGS="" bash scripts/r04_lay.sh && \
bash scripts/profile.sh walks 2 --tx layers9,opts5,forward2,build2,fields9 && \
bash scripts/profile.sh optsc5 2 --tx optsc5
