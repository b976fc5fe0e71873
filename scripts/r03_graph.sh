#!/bin/bash
# HIP-graph receive loops: the GPU tests, the C++ example at four ring shapes (eager and
# graph, parses on one stream or forked over 4), and the bench leg alone
set -o pipefail
O=gpurun_out/r03_graph
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_graphs.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 60 ./examples/rx_graph 4096 64 50 4 > $O/rx_graph_4k.log 2>&1 && \
timeout -k 10 60 ./examples/rx_graph 16384 64 50 4 > $O/rx_graph_16k.log 2>&1 && \
timeout -k 10 60 ./examples/rx_graph 65536 16 50 4 > $O/rx_graph_64k.log 2>&1 && \
timeout -k 10 60 ./examples/rx_graph 262144 4 50 4 > $O/rx_graph_256k.log 2>&1 && \
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --also "" --tx "" --compact "" --strong "" --opts "" --host "" --no-cpu --no-config1 > $O/bench.json 2> $O/bench.log
