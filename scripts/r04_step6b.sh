#!/bin/bash
# repeat of the step-6 A/B on the legs that moved
set -o pipefail
O=gpurun_out/r04_step6b
mkdir -p $O
run() { timeout -k 10 300 python3 -u tools/ab_lib.py ab/old/librpkt_gpu.so --rounds 9 --launches 20 "$@" >> $O/ab_old.jsonl 2>> $O/ab_old.log; }
run --leg parse3 && run --leg parsec11 --flags 11 && run --leg parse3 && run --leg parsec3 && \
run --leg parse11 --flags 11 && run --leg parse3 && run --leg popts5 || exit 1
echo done
