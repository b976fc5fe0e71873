#!/bin/bash
# round 3 profile refresh, part B: TX / walk legs; then the 2-rank gloo rehearsal of the
# weak, strong and sharded legs on the one GPU
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
bash "$R/scripts/profile.sh" walks 2 --tx layers9,opts5,forward2,build2,fields9
bash "$R/scripts/profile.sh" build3 2 --tx build3
bash "$R/scripts/profile.sh" optsc5 2 --tx optsc5
mkdir -p "$R/gpurun_out/r03_g2"
cd "$R" && timeout -k 10 600 python3 -u bench.py --gpus 2 --dist-backend gloo --also 4 --tx "" --compact "" \
    --opts "" --host "" --no-cpu --steps 10 > gpurun_out/r03_g2/bench_g2_gloo.json 2> gpurun_out/r03_g2/bench_g2_gloo.log
