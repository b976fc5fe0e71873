#!/bin/bash
# Round 2: multi-rank rehearsal on the one-GPU lease + the new C-ABI reduce tests, then
# the default bench.  Every GPU step under its own time limit, chained with &&.
set -o pipefail
mkdir -p gpurun_out
python3 -c "import os; print('cpu_count', os.cpu_count(), 'affinity', len(os.sched_getaffinity(0)))" > gpurun_out/r02_host.txt
cat /sys/fs/cgroup/cpu.max >> gpurun_out/r02_host.txt 2>&1
nproc >> gpurun_out/r02_host.txt
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_dist.py tests/test_gpu_parity.py -k "dist or ranks or rccl or flow_reduce or bench or cpp" -x -v --timeout 300 --timeout-method thread > gpurun_out/r02_pytest_dist.log 2>&1 && \
timeout -k 10 300 python3 -u bench.py --gpus 2 --dist-backend gloo --config 4 --also 2 --tx "" --steps 20 --warmup 5 > gpurun_out/r02_bench_g2_gloo.json 2> gpurun_out/r02_bench_g2_gloo.log && \
timeout -k 10 900 python3 -u bench.py > gpurun_out/r02_bench2.json 2> gpurun_out/r02_bench2.log
