#!/bin/bash
# Out-of-window IPv6 header reads as dword loads + IPv6/UDP headers kept in a 64-B
# window: GPU parity, then A (this build) against B (ab/old: the previous source)
set -o pipefail
O=gpurun_out/r04_step6
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ip6.py tests/test_gpu_chains_ip6.py tests/test_gpu_chains.py tests/test_gpu_parity.py tests/test_gpu_tx.py tests/test_gpu_opts.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
run() { timeout -k 10 300 python3 -u tools/ab_lib.py ab/old/librpkt_gpu.so --rounds 7 --launches 20 "$@" >> $O/ab_old.jsonl 2>> $O/ab_old.log; }
run --leg parse11 --flags 11 && run --leg parsec11 --flags 11 && run --leg parsec10 --flags 11 && \
run --leg parse10 --flags 11 && run --leg parse2 && run --leg parse3 && run --leg chains7 && \
run --leg parse11 --flags 11 && run --leg parsec10 --flags 11 || exit 1
echo done
