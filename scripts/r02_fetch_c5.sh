#!/bin/bash
# FETCH_SIZE per parse-kernel variant on config 5 (where does the 1.15x read over-fetch come from?)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/fetch_c5
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT" -o fetch \
    -- python3 "$R/tools/ablate.py" --configs 5,4,3 --variants 0,1,15,24,25,3 --rounds 1 --launches 4 > "$OUT/ablate.log" 2>&1
