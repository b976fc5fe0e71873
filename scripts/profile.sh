#!/bin/bash
# Profile pass for the GPU box: kernel trace + stats, then FETCH_SIZE and WRITE_SIZE
# in separate PMC passes (MI355X_MICROARCH.md §rocprofv3 PMC slots), for one bench
# config.  Usage:  bash scripts/profile.sh <tag> <config>
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; CFG=$2
OUT=$R/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
ARGS=(--no-cpu --config "$CFG" --also "" --tx "" --compact "" --strong "" --opts "" --ring "" --host "" --rx-graph "" --steps 20 --warmup 5 "${@:3}")
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$OUT" -o trace \
    -- python3 "$R/bench.py" "${ARGS[@]}" > "$OUT/trace_bench.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE -T --output-format csv -d "$OUT" -o fetch \
    -- python3 "$R/bench.py" "${ARGS[@]}" > "$OUT/fetch_bench.log" 2>&1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE -T --output-format csv -d "$OUT" -o write \
    -- python3 "$R/bench.py" "${ARGS[@]}" > "$OUT/write_bench.log" 2>&1
# read requests by size (TCC_EA0_RDREQ_{32B,64B,128B} + all: the 4 TCC slots): the exact
# read bytes, which calibrate FETCH_SIZE's x2 for access shapes other than streaming
timeout -k 10 400 rocprofv3 --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum \
    TCC_EA0_RDREQ_sum -T --output-format csv -d "$OUT" -o rdreq \
    -- python3 "$R/bench.py" "${ARGS[@]}" > "$OUT/rdreq_bench.log" 2>&1
echo "profile $TAG (config $CFG) done"
