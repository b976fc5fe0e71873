#!/bin/bash
# compact config-2 parse at batch sizes whose wave counts fill 2, 2.67 and 3 rounds of
# the device's resident slots (24 waves per CU): does the last partial round cost?
set -o pipefail
O=gpurun_out/r03_tail
mkdir -p $O
for n in 786432 1048576 1179648; do
  timeout -k 10 300 python3 -u bench.py --record compact --frames $n --steps 50 --warmup 10 --also "" --tx "" --compact "" --strong "" --opts "" --host "" --rx-graph "" --no-cpu --no-config1 > $O/c2c_$n.json 2> $O/c2c_$n.log || exit 1
done
