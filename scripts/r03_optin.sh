#!/bin/bash
# fused option walks run as the L4 stream's hook (in its first loads' shadow) vs before
# the stream; same process, outputs compared
set -o pipefail
O=gpurun_out/r03_optin
mkdir -p $O
for leg in popts5 poptsc5 popts3; do
  timeout -k 10 200 python3 -u tools/ab_lib.py rpkt_amd/_ab/optin/librpkt_gpu.so --leg $leg --rounds 7 >> $O/optin.log 2>&1 || exit 1
done
