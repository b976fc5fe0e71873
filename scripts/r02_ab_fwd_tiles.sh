#!/bin/bash
# forward: tiles per wave with the next tile's window prefetched (64-B-window compile)
set -o pipefail
mkdir -p gpurun_out/fwd_tiles
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_tx.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/fwd_tiles/tx_tests.log 2>&1 || exit 1
for b in t2 t4; do
  timeout -k 10 200 python3 -u tools/ab_lib.py rpkt_amd/_build_$b/librpkt_gpu.so --leg forward2 --rounds 8 --launches 24 \
    > gpurun_out/fwd_tiles/ab_forward2_$b.log 2>&1 || exit 1
done
timeout -k 10 200 python3 -u tools/ablate_fwd.py --variants 10,15,16,0,5 --rounds 6 \
    > gpurun_out/fwd_tiles/ablate_fwd.log 2>&1
