#!/bin/bash
# Turn a scripts/refresh_profiles.sh run (gpurun_out/prof_*) into the committed
# summaries under profiles/: traffic_c<cfg>.json / traffic_tx.json (read by bench.py)
# and per-profile trace stats, per-kernel PMC averages and bench logs.  Host side.
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
G=$R/gpurun_out
RND=${RND:-r02}
for t in ${TAGS:-c2 c3 c4 c5 c7 c10 c11 c2_compact c3_compact c11_compact c5_opts c5_opts_compact walks build3 optsc5 build11 forward10 opts11 tunnel13 encap13}; do
    P=$G/prof_$t; D=$R/profiles/${RND}_$t
    mkdir -p "$D"
    cp "$P/trace_kernel_stats.csv" "$P/trace_bench.log" "$D/"
    for k in fetch write rdreq; do
        [ -f "$P/${k}_counter_collection.csv" ] || continue
        [ -f "$P/${k}_bench.log" ] && cp "$P/${k}_bench.log" "$D/"
        python3 "$R/tools/pmc_by_kernel.py" "$P/${k}_counter_collection.csv" > "$D/${k}_by_kernel.json"
    done
    if [ "$t" = build3 ] || [ "$t" = optsc5 ] || [ "$t" = build11 ] || [ "$t" = forward10 ] ||
       [ "$t" = opts11 ] || [ "$t" = tunnel13 ] || [ "$t" = encap13 ]; then
        python3 "$R/tools/traffic.py" "$P" tx:$t "$R/profiles/traffic_tx.json"
    elif [ "$t" = walks ]; then
        python3 "$R/tools/traffic.py" "$P" tx "$R/profiles/traffic_tx.json"
    elif [ "${t%_compact}" != "$t" ] || [ "${t%_opts}" != "$t" ]; then
        c=${t#c}; python3 "$R/tools/traffic.py" "$P" "${c%%_*}" "$R/profiles/traffic_$t.json"
    else
        python3 "$R/tools/traffic.py" "$P" "${t#c}" "$R/profiles/traffic_$t.json"
    fi
done
