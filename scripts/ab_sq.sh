#!/bin/bash
# SQ counters (one PMC pass per side, kernel trace off) of one ab_lib leg, side A (in-tree
# build) and side B (a --build library): VALU instructions and wait cycles per wave of
# the kernel named <kernel>, into gpurun_out/absq_<tag>/summary.json.
#   bash scripts/ab_sq.sh <tag> <lib_b.so> <kernel> "<ab_lib args>"
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; LIB=$(cd "$R" && realpath "$2"); KERNEL=$3; ARGS=$4
OUT=$R/gpurun_out/absq_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
COUNTERS=${COUNTERS:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS}
for side in A B; do
    timeout -s KILL 120 rocprofv3 --pmc $COUNTERS -T --output-format csv -d "$OUT" -o ${side}_sq \
        -- python3 "$R/tools/ab_lib.py" "$LIB" --sides $side --rounds 3 --launches 10 $ARGS \
        > "$OUT/${side}.log" 2>&1
done
python3 - "$OUT" "$KERNEL" <<'PY'
import collections, csv, glob, json, sys
out, kernel = sys.argv[1], sys.argv[2]
res = {}
for side in "AB":
    f = glob.glob("%s/%s_sq_counter_collection.csv" % (out, side)) or \
        glob.glob("%s/**/%s_sq_counter_collection.csv" % (out, side), recursive=True)
    rows = list(csv.DictReader(open(f[0])))
    agg = collections.defaultdict(list)
    for r in rows:
        if kernel in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {k: sum(v) / len(v) for k, v in agg.items()}
    w = m.get("SQ_WAVES") or 1
    m["valu_per_wave"] = m.get("SQ_ACTIVE_INST_VALU", 0) / w
    m["wait_any_frac"] = m.get("SQ_WAIT_ANY", 0) / max(1, m.get("SQ_WAVE_CYCLES", 1))
    m["launches"] = len(agg.get("SQ_WAVES", []))
    res[side] = m
json.dump(res, open(out + "/summary.json", "w"), indent=1)
print(json.dumps({s: {k: round(v, 3) for k, v in res[s].items() if k in ("valu_per_wave", "wait_any_frac", "SQ_WAVES")} for s in res}))
PY
