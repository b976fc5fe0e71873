#!/bin/bash
# header-only 80-B-record parse of short strided frames on the 64-B-window compile too?
# A (this build: 128-B windows) against B (ab/full64all)
set -o pipefail
O=gpurun_out/r04_step9b
mkdir -p $O
run() { timeout -k 10 300 python3 -u tools/ab_lib.py ab/full64all/librpkt_gpu.so --rounds 9 --launches 20 "$@" >> $O/ab.jsonl 2>> $O/ab.log; }
run --leg parse2 && run --leg parse2 && run --leg parse2 && run --leg parse10 --flags 11 || exit 1
echo done
