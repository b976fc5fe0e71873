#!/bin/bash
# full-record config-2 parse at three batch sizes: the fixed per-launch cost
set -o pipefail
O=gpurun_out/r03_tail
mkdir -p $O
for n in 786432 1048576 1572864; do
  timeout -k 10 300 python3 -u bench.py --frames $n --steps 50 --warmup 10 --also "" --tx "" --compact "" --strong "" --opts "" --host "" --rx-graph "" --no-cpu --no-config1 > $O/c2_$n.json 2> $O/c2_$n.log || exit 1
done
