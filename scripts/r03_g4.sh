#!/bin/bash
# 4-rank rehearsal of the distributed bench on the one GPU (gloo: RCCL needs one GPU per
# rank): weak (configs 2/3), strong (config 2/3 split, config 4 sharded + counter reduce)
set -o pipefail
O=gpurun_out/r03_g4
mkdir -p $O
timeout -k 10 900 python3 -u bench.py --gpus 4 --dist-backend gloo --also 3,4 --tx "" --compact "" \
    --opts "" --host "" --rx-graph "" --no-cpu --steps 10 > $O/bench_g4_gloo.json 2> $O/bench_g4_gloo.log
