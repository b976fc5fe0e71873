#!/bin/bash
# field getters: the block's layer records as coalesced loads through LDS (A) vs one
# 64-B record per lane from global memory (B: _build_recglobal)
set -o pipefail
OUT=gpurun_out/ab_frec
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fields.py -x -q --timeout 120 --timeout-method thread \
    > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/ab_lib.py rpkt_amd/_build_recglobal/librpkt_gpu.so --leg fields9 --rounds 8 --launches 20 \
    > $OUT/ab_fields9.log 2>&1
