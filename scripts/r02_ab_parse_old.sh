#!/bin/bash
# same-process A/B: the parse kernel of the current build vs commit fa19e07's
set -o pipefail
mkdir -p gpurun_out/ab_fa19
for leg in parse5 parse3 parse2; do
  timeout -k 10 300 python3 -u tools/ab_lib.py rpkt_amd/_build_fa19/librpkt_gpu.so --leg $leg --rounds 6 --launches 16 \
    > gpurun_out/ab_fa19/ab_$leg.log 2>&1 || exit 1
done
