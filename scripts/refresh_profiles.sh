#!/bin/bash
# Refresh the rocprofv3 trace + PMC traffic summaries the bench line cites, for the
# current engine build (GPU box).  Stops at the first failing pass.
#   bash scripts/refresh_profiles.sh [tag ...]   (default: every tag below)
#   -> gpurun_out/prof_<tag>/, collected on the host by scripts/collect_profiles.sh
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
ALL="c2 c3 c4 c5 c7 c10 c11 c2_compact c3_compact c11_compact c5_opts c5_opts_compact walks build3 optsc5 build11 forward10 opts11 tunnel13 encap13"
for t in ${@:-$ALL}; do
    case $t in
        c2|c3|c4|c5|c7|c10|c11) bash "$R/scripts/profile.sh" "$t" "${t#c}" ;;
        c5_opts) bash "$R/scripts/profile.sh" c5_opts 5 --main-opts ;;
        c5_opts_compact) bash "$R/scripts/profile.sh" c5_opts_compact 5 --main-opts --record compact ;;
        c*_compact) c=${t#c}; bash "$R/scripts/profile.sh" "$t" "${c%_compact}" --record compact ;;
        walks) bash "$R/scripts/profile.sh" walks 2 --tx layers9,opts5,forward2,build2,fields9 ;;
        build3|optsc5|build11|forward10|opts11|tunnel13|encap13) bash "$R/scripts/profile.sh" "$t" 2 --tx "$t" ;;
        *) echo "unknown tag $t"; exit 2 ;;
    esac
done
