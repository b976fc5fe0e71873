#!/bin/bash
# compact parse of short strided frames through the 64-B-window compile (A) vs the
# 128-B-window kernel (B: _build_w64off, -DRPKT_PARSE_W64_ON=0); parity tests first
set -o pipefail
OUT=gpurun_out/ab_parsec_w64
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q -k "compact or short_strided" --timeout 120 --timeout-method thread \
    > $OUT/tests.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/ab_lib.py rpkt_amd/_build_w64off/librpkt_gpu.so --leg parsec2 --rounds 8 --launches 20 \
    > $OUT/ab_parsec2.log 2>&1 || exit 1
timeout -k 10 200 python3 -u tools/ab_lib.py rpkt_amd/_build_w64off/librpkt_gpu.so --leg parse2 --rounds 8 --launches 20 \
    > $OUT/ab_parse2.log 2>&1
