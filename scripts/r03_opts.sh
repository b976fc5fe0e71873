#!/bin/bash
# fused parse + option walks: parity tests, a config-5 bench beside the two-kernel path,
# and a kernel trace of the fused leg
set -o pipefail
O=gpurun_out/r03_opts
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_opts.py -x -v --timeout 120 --timeout-method thread > $O/pytest_opts.log 2>&1 && \
timeout -k 10 400 python3 -u bench.py --config 5 --also "" --tx "opts5,optsc5" --compact "" --opts 5 --no-cpu --no-config1 --steps 20 > $O/bench.json 2> $O/bench.log && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -T --output-format csv -d $GRAFT_REPO_ROOT/$O/trace -o trace -- python3 $GRAFT_REPO_ROOT/bench.py --config 5 --main-opts --also "" --tx "" --compact "" --opts "" --no-cpu --no-config1 --steps 20 > $GRAFT_REPO_ROOT/$O/trace.log 2>&1
