#!/bin/bash
# A/B timing of a B-side build (python tools/ab_lib.py --build ab/<name> -D...) against the
# in-tree library on bench legs, outputs compared byte for byte, one JSON line per leg
# into gpurun_out/ab_<tag>/ab.jsonl.  Stops at the first failing leg.
#   bash scripts/ab_run.sh <tag> <lib_b.so> "<ab_lib args>" ["<ab_lib args>" ...]
#   e.g. bash scripts/ab_run.sh joint ab/nojoint/librpkt_gpu.so "--leg parse3" "--leg parse11 --flags 11"
set -o pipefail
TAG=$1; LIB=$2; shift 2
O=gpurun_out/ab_$TAG
mkdir -p "$O"
for legargs in "$@"; do
    timeout -k 10 300 python3 -u tools/ab_lib.py "$LIB" --rounds 9 --launches 20 $legargs \
        >> "$O/ab.jsonl" 2>> "$O/ab.log" || exit 1
done
echo done
