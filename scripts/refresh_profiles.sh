#!/bin/bash
# Refresh every rocprofv3 trace + PMC traffic summary the bench line cites, for the
# current engine build (GPU box).  Stops at the first failing pass.
#   bash scripts/refresh_profiles.sh        -> gpurun_out/prof_{c2,c3,c4,c5,c7,c*_compact,c5_opts*,walks,build3,optsc5}
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
for c in 2 3 4 5 7; do
    bash "$R/scripts/profile.sh" "c$c" "$c"
done
for c in 2 3; do
    bash "$R/scripts/profile.sh" "c${c}_compact" "$c" --record compact
done
bash "$R/scripts/profile.sh" c5_opts 5 --main-opts
bash "$R/scripts/profile.sh" c5_opts_compact 5 --main-opts --record compact
bash "$R/scripts/profile.sh" walks 2 --tx layers9,opts5,forward2,build2,fields9
bash "$R/scripts/profile.sh" build3 2 --tx build3
bash "$R/scripts/profile.sh" optsc5 2 --tx optsc5
