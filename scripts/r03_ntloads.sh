#!/bin/bash
# read-once loads non-temporal: flow events in the histogram (B: -DRPKT_FLOW_EV_NT=0) and
# packed frame offsets (B: -DRPKT_SPAN_NT=0); same process, outputs compared
set -o pipefail
O=gpurun_out/r03_ntloads
mkdir -p $O
timeout -k 10 150 python3 -u tools/ab_lib.py rpkt_amd/_ab/evdef/librpkt_gpu.so --leg flow4 --rounds 9 > $O/ab_flow.log 2>&1 && \
timeout -k 10 150 python3 -u tools/ab_lib.py rpkt_amd/_ab/spandef/librpkt_gpu.so --leg parse4 --rounds 5 > $O/ab_span.log 2>&1 && \
timeout -k 10 150 python3 -u tools/ab_lib.py rpkt_amd/_ab/spandef/librpkt_gpu.so --leg parse5 --rounds 5 >> $O/ab_span.log 2>&1 && \
timeout -k 10 150 python3 -u tools/ab_lib.py rpkt_amd/_ab/spandef/librpkt_gpu.so --leg layers9 --rounds 9 >> $O/ab_span.log 2>&1 && \
timeout -k 10 150 python3 -u tools/ab_lib.py rpkt_amd/_ab/spandef/librpkt_gpu.so --leg popts5 --rounds 5 >> $O/ab_span.log 2>&1
