#!/bin/bash
# L4 stream owners from marks on short-range tiles (A, product) against the cursor with
# binary search everywhere (B: -DRPKT_STREAM_MARKS=0); the full GPU suite first
set -o pipefail
O=gpurun_out/r03_marks
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
for leg in parse4 parse5 parse3 popts5 poptsc5 build3; do
  timeout -k 10 200 python3 -u tools/ab_lib.py rpkt_amd/_ab/nomarks/librpkt_gpu.so --leg $leg --rounds 5 >> $O/ab.log 2>&1 || exit 1
done
