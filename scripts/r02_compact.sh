#!/bin/bash
# compact records: GPU parity, host-inclusive rates for both record sizes, bench legs
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -k compact -x -v --timeout 120 --timeout-method thread > gpurun_out/r02_pytest_compact.log 2>&1 && \
timeout -k 10 300 python3 -u tools/host_rate.py > gpurun_out/r02_host_rate.log 2>&1 && \
timeout -k 10 300 python3 -u bench.py --also "" --tx "" --no-cpu --compact 2,3 > gpurun_out/r02_bench_compact.json 2> gpurun_out/r02_bench_compact.log
