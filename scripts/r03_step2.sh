#!/bin/bash
# run-then-TLV walk steps: parity, then A/B against one-thing-per-step, fused + standalone;
# the compact parse alone for the fused compact leg's ratio
set -o pipefail
O=gpurun_out/r03_step2
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_opts.py -x -q --timeout 170 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for leg in popts5 poptsc5 opts5 optsc5 parsec5 parse5; do
  timeout -k 10 300 python3 -u tools/ab_lib.py rpkt_amd/_ab/step1/librpkt_gpu.so --leg $leg --rounds 7 >> $O/ab_step1.log 2>&1 || exit 1
done
