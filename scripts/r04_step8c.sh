#!/bin/bash
# the 64-KB-gated joint loader: parity, then A/B against the separate edge pass
set -o pipefail
O=gpurun_out/r04_step8c
mkdir -p $O
timeout -k 10 700 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_ip6.py tests/test_gpu_ring.py tests/test_gpu_opts.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
run() { timeout -k 10 300 python3 -u tools/ab_lib.py ab/nojoint/librpkt_gpu.so --rounds 9 --launches 10 "$@" >> $O/ab.jsonl 2>> $O/ab.log; }
run --leg parse5 && run --leg parse3 && run --leg parse11 --flags 11 && run --leg popts5 && run --leg parsec3 && run --leg parse5 || exit 1
echo done
