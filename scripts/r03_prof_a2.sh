#!/bin/bash
# round 3 profile refresh after the parse_ring change, part A2: compact and fused legs
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
for c in 2 3; do
    bash "$R/scripts/profile.sh" "c${c}_compact" "$c" --record compact
done
bash "$R/scripts/profile.sh" c5_opts 5 --main-opts
bash "$R/scripts/profile.sh" c5_opts_compact 5 --main-opts --record compact
