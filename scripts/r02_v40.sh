#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out/v40
timeout -k 10 300 python3 -u tools/variant_check.py --variants 40,41,42,43 > gpurun_out/v40/check.log 2>&1 && \
timeout -k 10 300 python3 -u tools/ablate.py --configs 5,3,4 --variants 0,40,41,42,43 --rounds 4 --launches 10 > gpurun_out/v40/ablate.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/gpurun_out/v40" -o fetch \
    -- python3 "$R/tools/ablate.py" --configs 5,3,4 --variants 0,41,42,43 --rounds 1 --launches 3 > "$R/gpurun_out/v40/fetch_ablate.log" 2>&1
