#!/bin/bash
# PMC passes (FETCH_SIZE, then WRITE_SIZE: separate runs) of one ab_lib leg, side A
# (in-tree build) and side B (a --build library), into gpurun_out/abpmc_<tag>/.
#   bash scripts/ab_pmc.sh <tag> <lib_b.so> "<ab_lib args>"
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; LIB=$(cd "$R" && realpath "$2"); ARGS=$3
OUT=$R/gpurun_out/abpmc_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for side in A B; do
    for c in FETCH_SIZE WRITE_SIZE; do
        timeout -k 10 300 rocprofv3 --pmc $c -T --output-format csv -d "$OUT" -o ${side}_$c \
            -- python3 "$R/tools/ab_lib.py" "$LIB" --sides $side --rounds 3 --launches 10 $ARGS \
            > "$OUT/${side}_$c.log" 2>&1
    done
done
echo "abpmc $TAG done"
