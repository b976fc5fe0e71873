#!/bin/bash
# 8-rank rehearsal of bench.py's own launcher on the one leased GPU (gloo), config 4
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u bench.py --gpus 8 --dist-backend gloo --config 4 --also "" --tx "" --compact "" --frames 800000 --steps 5 --warmup 2 --min-warmup-s 0 > gpurun_out/r02_bench_g8_gloo.json 2> gpurun_out/r02_bench_g8_gloo.log
