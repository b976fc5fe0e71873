#!/bin/bash
# SQ stall breakdown of one kernel (one PMC pass, kernel trace off): where do waves
# spend their cycles?  Usage: [COUNTERS="..."] bash scripts/sq_counters.sh <tag> <config> [kernel] [bench args]
# (at most 8 SQ_ counters per pass)
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; CFG=$2; KERNEL=${3:-parse_kernel}
OUT=$R/gpurun_out/sq_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
COUNTERS=${COUNTERS:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS}
timeout -s KILL 120 rocprofv3 --pmc $COUNTERS \
    -T --output-format csv -d "$OUT" -o sq \
    -- python3 "$R/bench.py" --no-cpu --config "$CFG" --also "" --tx "" --compact "" --strong "" --opts "" --host "" --rx-graph "" --steps 10 --warmup 2 --min-warmup-s 0 "${@:4}" > "$OUT/bench.log" 2>&1
python3 - "$OUT" "$KERNEL" <<'PY'
import csv, collections, sys, json
rows = list(csv.DictReader(open(sys.argv[1] + "/sq_counter_collection.csv")))
agg = collections.defaultdict(list)
for r in rows:
    if r["Kernel_Name"].startswith(sys.argv[2]):
        agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
print(json.dumps({k: sum(v[2:]) / max(1, len(v[2:])) for k, v in agg.items()}))
PY
