#!/bin/bash
# field getters: a request on the same (protocol, nth) as the one before reuses its layer
# search (A) vs a search per request (B: _build_nosame); field GPU tests first
set -o pipefail
OUT=gpurun_out/ab_samelayer
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_fields.py -x -q --timeout 120 --timeout-method thread \
    > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/ab_lib.py rpkt_amd/_build_nosame/librpkt_gpu.so --leg fields9 --rounds 8 --launches 20 \
    > $OUT/ab_fields9.log 2>&1
