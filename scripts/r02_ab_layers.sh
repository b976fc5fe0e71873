#!/bin/bash
# same-process A/B of the layer walk: in-tree build (A) vs rpkt_amd/_build_head (B)
set -o pipefail
mkdir -p gpurun_out/ab_layers
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_layers.py -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/ab_layers/tests.log 2>&1 || exit 1
for leg in layers9 layers2 layers5; do
  timeout -k 10 200 python3 -u tools/ab_lib.py rpkt_amd/_build_head/librpkt_gpu.so --leg $leg --rounds 8 --launches 20 \
    > gpurun_out/ab_layers/ab_${leg}_${TAG:-x}.log 2>&1 || exit 1
done
