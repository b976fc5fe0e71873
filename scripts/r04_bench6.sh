#!/bin/bash
# first measurement of the dual-stack legs (configs 10, 11) and the 8-slot ring leg, then
# rocprofv3 trace + FETCH/WRITE passes for configs 10 and 11
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r04_bench6
mkdir -p $O
timeout -k 10 400 python3 -u bench.py --config 11 --also 10 --tx "" --compact 10,11 --strong "" --opts "" --host "" --rx-graph "" --no-config1 --ring 2 --cpu-seconds 5 > $O/bench.json 2> $O/bench.log && \
bash scripts/profile.sh c10 10 && bash scripts/profile.sh c11 11
