#!/bin/bash
# In-window L4 instantiation for strided batches of short frames: parity, then A (this
# build) against B (ab/old: the previous source)
set -o pipefail
O=gpurun_out/r04_step7
mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ip6.py tests/test_gpu_ring.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
run() { timeout -k 10 300 python3 -u tools/ab_lib.py ab/old/librpkt_gpu.so --rounds 7 --launches 20 "$@" >> $O/ab_old.jsonl 2>> $O/ab_old.log; }
run --leg parse10 --flags 11 && run --leg parsec10 --flags 11 && run --leg parse2 --flags 3 && \
run --leg parsec2 --flags 3 && run --leg ring2 --flags 3 && run --leg ringc2 --flags 3 && \
run --leg parse2 && run --leg parse3 && run --leg parse10 --flags 11 || exit 1
echo done
