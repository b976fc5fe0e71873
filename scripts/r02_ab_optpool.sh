#!/bin/bash
# option walks from compact records with a pool of 256 frames per wave (A) vs one
# 64-frame tile per wave (B: _build_nopool, -DRPKT_OPT_POOL=0); the full-record walk
# after the step refactor vs the previous commit (B: _build_prev)
set -o pipefail
OUT=gpurun_out/ab_optpool
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_opts.py -x -q --timeout 120 --timeout-method thread \
    > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/ab_lib.py rpkt_amd/_build_nopool/librpkt_gpu.so --leg optsc5 --rounds 8 --launches 20 \
    > $OUT/ab_optsc5.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/ab_lib.py rpkt_amd/_build_prev/librpkt_gpu.so --leg opts5 --rounds 8 --launches 20 \
    > $OUT/ab_opts5_prev.log 2>&1
