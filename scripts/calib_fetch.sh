#!/bin/bash
# FETCH_SIZE calibration on config 3: product kernel (nt stream), default-policy
# stream variant, and the pure streaming read reference over the same buffer.
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$R/gpurun_out/calib
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d "$OUT" -o fetch \
    -- python3 "$R/tools/ablate.py" --configs 3 --rounds 2 --launches 5 --variants 0,22,14,3 \
    > "$OUT/fetch.log" 2>&1
python3 "$R/tools/pmc_by_kernel.py" "$OUT/fetch_counter_collection.csv" > "$OUT/fetch_by_kernel.json"
echo calib done
