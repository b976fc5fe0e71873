#!/bin/bash
# field getters after the same-layer reuse: 16 requests in flight (A) vs 8 (B: _build_fg8)
set -o pipefail
OUT=gpurun_out/ab_fg8b
mkdir -p $OUT
timeout -k 10 200 python3 -u tools/ab_lib.py rpkt_amd/_build_fg8/librpkt_gpu.so --leg fields9 --rounds 8 --launches 20 \
    > $OUT/ab_fields9.log 2>&1
