#!/bin/bash
# forward's write-back store policy: sc0|nt (A, product) against nt (B: -DRPKT_FWD_WB_AUX=2)
# and sc0 (-DRPKT_FWD_WB_AUX=1); same process, outputs compared
set -o pipefail
O=gpurun_out/r03_fwdwb
mkdir -p $O
timeout -k 10 150 python3 -u tools/ab_lib.py rpkt_amd/_ab/wb2/librpkt_gpu.so --leg forward2 --rounds 9 > $O/ab.log 2>&1 && \
timeout -k 10 150 python3 -u tools/ab_lib.py rpkt_amd/_ab/wb1/librpkt_gpu.so --leg forward2 --rounds 9 >> $O/ab.log 2>&1
