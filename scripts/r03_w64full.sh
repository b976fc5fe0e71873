#!/bin/bash
# config 2 parse with 80-B records: the 64-B-window compile (A, code since removed) against the
# 128-B windows (B: -DRPKT_PARSE_W64_FULL_ON=0); same process, outputs compared
set -o pipefail
O=gpurun_out/r03_w64full
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_parity.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 150 python3 -u tools/ab_lib.py rpkt_amd/_ab/w128full/librpkt_gpu.so --leg parse2 --rounds 9 >> $O/ab.log 2>&1 || exit 1
done
