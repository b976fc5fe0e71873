#!/bin/bash
# compact rings of short strided frames on the 64-B-window compile: the ring tests, the
# full GPU suite, then the bench's receive-loop leg (ring_compact mode) against a build
# with the 64-B-window dispatch off (B: -DRPKT_PARSE_W64_ON=0, via bench_with_lib)
set -o pipefail
O=gpurun_out/r03_ringw64
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || exit 1
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --also "" --tx "" --compact "" --strong "" --opts "" --host "" --no-cpu --no-config1 > $O/bench_A.json 2> $O/bench_A.log || exit 1
timeout -k 10 300 python3 -u tools/bench_with_lib.py rpkt_amd/_ab/ringw128/librpkt_gpu.so --steps 20 --warmup 5 --also "" --tx "" --compact "" --strong "" --opts "" --host "" --no-cpu --no-config1 > $O/bench_B.json 2> $O/bench_B.log
