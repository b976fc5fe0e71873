#!/bin/bash
# Ring launch at 1 wave per block against the product's 4, then the whole GPU suite
set -o pipefail
O=gpurun_out/r04_step5
mkdir -p $O
for leg in ring2 ringc2 ring2 ringc2; do
  timeout -k 10 300 python3 -u tools/ab_lib.py ab/ring1/librpkt_gpu.so --leg $leg --rounds 7 --launches 10 \
      >> $O/ab_ring1.jsonl 2>> $O/ab_ring1.log || exit 1
done
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
echo done
