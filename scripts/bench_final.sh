#!/bin/bash
# End-of-round measurement pass: smoke, the default bench line (what the driver runs), and
# the rocprofv3 kernel-trace --stats summary of the bench's main leg.
#   bash scripts/bench_final.sh <round tag, e.g. r06>   -> gpurun_out/<tag>_bench/
set -o pipefail
O=gpurun_out/${1:-r06}_bench
mkdir -p $O
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 900 python3 -u bench.py --detail $O/bench_detail.json > $O/bench.json 2> $O/bench.log || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T --output-format csv -d "$GRAFT_REPO_ROOT/$O/prof" -o main \
    -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu --also "" --tx "" --compact "" --strong "" --opts "" \
       --host "" --rx-graph "" --ring "" > "$GRAFT_REPO_ROOT/$O/prof_bench.json" 2> "$GRAFT_REPO_ROOT/$O/prof_bench.log" || exit 1
echo done
