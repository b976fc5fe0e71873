#!/bin/bash
# build_kernel's record loads non-temporal (A, product) against default policy (B:
# -DRPKT_BUILD_REC_NT=0); same process, outputs compared; the TX GPU tests
set -o pipefail
O=gpurun_out/r03_recnt
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_tx.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_tx.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 150 python3 -u tools/ab_lib.py rpkt_amd/_ab/recdef/librpkt_gpu.so --leg build2 --rounds 9 >> $O/ab.log 2>&1 || exit 1
done
timeout -k 10 150 python3 -u tools/ab_lib.py rpkt_amd/_ab/recdef/librpkt_gpu.so --leg build3 --rounds 5 >> $O/ab.log 2>&1
