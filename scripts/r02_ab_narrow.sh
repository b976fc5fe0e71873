#!/bin/bash
# field getters: fields of <= 32 bits take two loads and 32-bit math (A, code since
# removed) vs three loads and the 64-bit path for every field (B: _build_wide)
set -o pipefail
OUT=gpurun_out/ab_narrow
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fields.py -x -q --timeout 120 --timeout-method thread \
    > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/ab_lib.py rpkt_amd/_build_wide/librpkt_gpu.so --leg fields9 --rounds 8 --launches 20 \
    > $OUT/ab_fields9.log 2>&1
