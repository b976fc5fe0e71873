#!/bin/bash
# 80-B-record L4 parse of short strided frames on the 64-B-window compile: parity, then
# A (this build) against B (ab/nofull64: the 128-B-window in-window instantiation)
set -o pipefail
O=gpurun_out/r04_step9
mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ip6.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
run() { timeout -k 10 300 python3 -u tools/ab_lib.py ab/nofull64/librpkt_gpu.so --rounds 9 --launches 20 "$@" >> $O/ab.jsonl 2>> $O/ab.log; }
run --leg parse10 --flags 11 && run --leg parse2 --flags 3 && run --leg parse2 && run --leg parse10 --flags 11 && run --leg parse2 --flags 3 || exit 1
echo done
