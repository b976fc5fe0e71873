#!/bin/bash
# final state of round 2: GPU suite, smoke, the profiles of the units changed since the
# last full refresh (walk legs incl. fields; options from compact records), default bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r02_pytest_gpu.log 2>&1 && \
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02_smoke.log 2>&1 && \
bash scripts/profile.sh walks 2 --tx layers9,opts5,forward2,build2,fields9 > gpurun_out/r02_prof_walks.log 2>&1 && \
bash scripts/profile.sh optsc5 2 --tx optsc5 > gpurun_out/r02_prof_optsc5.log 2>&1 && \
timeout -k 10 900 python3 -u bench.py > gpurun_out/r02_bench_final.json 2> gpurun_out/r02_bench_final.log
