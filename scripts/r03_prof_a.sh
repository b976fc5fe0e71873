#!/bin/bash
# round 3 profile refresh, part A: parse legs (kernel trace + FETCH_SIZE + WRITE_SIZE)
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
