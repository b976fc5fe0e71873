#!/bin/bash
# repeat of the joint-loader A/B on config 5 (and 4, 3 as controls)
set -o pipefail
O=gpurun_out/r04_step8b
mkdir -p $O
run() { timeout -k 10 300 python3 -u tools/ab_lib.py ab/nojoint/librpkt_gpu.so --rounds 9 --launches 10 "$@" >> $O/ab.jsonl 2>> $O/ab.log; }
run --leg parse5 && run --leg parse4 && run --leg parse5 && run --leg parse3 && run --leg parse5 || exit 1
echo done
