#!/bin/bash
# paired option walks: parity, then same-process A/B against the two-walks-per-step form;
# the multi-rank / threaded flow tests on the new build
set -o pipefail
O=gpurun_out/r03_paired
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_opts.py tests/test_gpu_dist.py -x -v --timeout 170 --timeout-method thread > $O/pytest.log 2>&1 && \
for leg in popts5 poptsc5 opts5 optsc5; do
  timeout -k 10 300 python3 -u tools/ab_lib.py rpkt_amd/_ab/unpaired/librpkt_gpu.so --leg $leg >> $O/ab.log 2>&1 || exit 1
done
