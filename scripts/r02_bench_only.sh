#!/bin/bash
# the default bench line on the current build
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u bench.py > gpurun_out/r02_bench_final2.json 2> gpurun_out/r02_bench_final2.log
