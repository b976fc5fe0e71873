#!/bin/bash
# IPv6 decode-and-verify: the new GPU parity tests, then the parse/opts/ring/tx suites
set -o pipefail
O=gpurun_out/r04_ip6
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ip6.py -x -v --timeout 200 --timeout-method thread > $O/pytest_ip6.log 2>&1 && \
timeout -k 10 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_opts.py tests/test_gpu_ring.py tests/test_gpu_tx.py tests/test_gpu_chains.py -x -q --timeout 200 --timeout-method thread > $O/pytest_regress.log 2>&1
