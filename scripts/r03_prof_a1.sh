#!/bin/bash
# round 3 profile refresh after the parse_ring change, part A1: the five parse configs
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
for c in 2 3 4 5 7; do
    bash "$R/scripts/profile.sh" "c$c" "$c"
done
