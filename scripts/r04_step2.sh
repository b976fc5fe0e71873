#!/bin/bash
# IPv6 option walks + owned communicator + ABI, then the launch-overlap probe
set -o pipefail
O=gpurun_out/r04_step2
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_ip6.py tests/test_gpu_opts.py tests/test_gpu_dist.py tests/test_abi.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 && \
timeout -k 10 200 python3 -u tools/overlap_probe.py > $O/probe.json 2> $O/probe.log && \
timeout -k 10 200 python3 -u tools/launch_stamps.py > $O/stamps.json 2> $O/stamps.log && \
timeout -k 10 200 python3 -u tools/launch_stamps.py --n 786432 > $O/stamps_075.json 2>> $O/stamps.log
