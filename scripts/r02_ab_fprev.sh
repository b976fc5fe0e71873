#!/bin/bash
# field getters: group-staged rows with shift row index (A) vs the previous commit (B:
# _build_prev, full-row stage indexed by a division by n_req), same process
set -o pipefail
OUT=gpurun_out/ab_fprev
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fields.py tests/test_gpu_layers.py -x -q --timeout 120 --timeout-method thread \
    > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/ab_lib.py rpkt_amd/_build_prev/librpkt_gpu.so --leg fields9 --rounds 8 --launches 20 \
    > $OUT/ab_prev.log 2>&1
