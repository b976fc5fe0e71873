#!/bin/bash
# Profile pass for the GPU box: kernel trace + stats, then FETCH_SIZE and WRITE_SIZE
# in separate PMC passes (MI355X_MICROARCH.md §rocprofv3 PMC slots).  Usage:
#   bash scripts/profile.sh <tag> [bench args...]
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT" -o trace \
    -- python3 "$R/bench.py" --no-cpu "$@" > "$OUT/trace_bench.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d "$OUT" -o fetch \
    -- python3 "$R/bench.py" --no-cpu --steps 5 --warmup 1 "$@" > "$OUT/fetch_bench.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d "$OUT" -o write \
    -- python3 "$R/bench.py" --no-cpu --steps 5 --warmup 1 "$@" > "$OUT/write_bench.log" 2>&1
echo "profile $TAG done"
