#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/txw64
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_tx.py -x -q --timeout 120 --timeout-method thread > gpurun_out/txw64/pytest.log 2>&1 && \
timeout -k 10 200 python3 -u tools/ab_lib.py rpkt_amd/_build_b/librpkt_gpu.so --leg forward2 > gpurun_out/txw64/ab_forward2.log 2>&1 && \
timeout -k 10 200 python3 -u tools/ab_lib.py rpkt_amd/_build_b/librpkt_gpu.so --leg build2 > gpurun_out/txw64/ab_build2.log 2>&1 && \
timeout -k 10 200 python3 -u tools/ablate_fwd.py --variants 9,10,1,11 --rounds 6 > gpurun_out/txw64/ablate_fwd.log 2>&1
