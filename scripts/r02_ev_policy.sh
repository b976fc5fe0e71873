#!/bin/bash
# config 4 step (parse with flow events + flow counters): nt event stores (product) vs default
set -o pipefail
OUT=gpurun_out/ev_policy
mkdir -p $OUT
ARGS=(--no-cpu --no-config1 --config 4 --also "" --tx "" --compact "" --steps 50)
for r in 1 2; do
  for lib in _build _build_evdef; do
    timeout -k 10 300 python3 -u tools/bench_with_lib.py rpkt_amd/$lib/librpkt_gpu.so "${ARGS[@]}" \
      > $OUT/${lib}_$r.json 2> $OUT/${lib}_$r.log || exit 1
  done
done
