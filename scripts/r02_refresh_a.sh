#!/bin/bash
# parse-unit profiles after the flow-histogram change, part 1 (configs 2, 3, 4, 2 compact)
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
for c in 2 3 4; do bash "$R/scripts/profile.sh" "c$c" "$c"; done
bash "$R/scripts/profile.sh" c2_compact 2 --record compact
