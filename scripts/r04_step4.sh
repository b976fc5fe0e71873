#!/bin/bash
# IPv6 over mbuf chains (GPU parity), then the parse at 1 / 2 waves per block against
# the product's 4 (tools/ab_lib.py, same process, outputs compared byte for byte)
set -o pipefail
O=gpurun_out/r04_step4
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_chains_ip6.py tests/test_gpu_chains.py tests/test_gpu_ip6.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for B in wpb1 wpb2; do
  for leg in parse2 parsec2 parse3 popts5 parse2 parsec2; do
    timeout -k 10 300 python3 -u tools/ab_lib.py ab/$B/librpkt_gpu.so --leg $leg --rounds 7 --launches 20 \
        >> $O/ab_$B.jsonl 2>> $O/ab_$B.log || exit 1
  done
done
echo done
