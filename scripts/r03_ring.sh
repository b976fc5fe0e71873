#!/bin/bash
# rpkt_gpu_parse_ring: parity tests, the graph tests, the C++ receive loop (eager / graph x
# one stream / 4 streams / ring call) at four ring shapes, the bench leg alone, and an A/B
# of the headline parse against the build before parse_tile was factored out
set -o pipefail
O=gpurun_out/r03_ring
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_ring.py tests/test_gpu_graphs.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 60 ./examples/rx_graph 4096 64 50 4 > $O/rx_graph_4k.log 2>&1 && \
timeout -k 10 60 ./examples/rx_graph 16384 64 50 4 > $O/rx_graph_16k.log 2>&1 && \
timeout -k 10 60 ./examples/rx_graph 65536 16 50 4 > $O/rx_graph_64k.log 2>&1 && \
timeout -k 10 60 ./examples/rx_graph 262144 4 50 4 > $O/rx_graph_256k.log 2>&1 && \
timeout -k 10 150 python3 -u tools/ab_lib.py rpkt_amd/_ab/pretile/librpkt_gpu.so --leg parse2 --rounds 9 > $O/ab_parse2.log 2>&1 && \
timeout -k 10 150 python3 -u tools/ab_lib.py rpkt_amd/_ab/pretile/librpkt_gpu.so --leg parse3 --rounds 5 >> $O/ab_parse2.log 2>&1 && \
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --also "" --tx "" --compact "" --strong "" --opts "" --host "" --no-cpu --no-config1 > $O/bench.json 2> $O/bench.log
