#!/bin/bash
# profile refresh of the TX / walk legs only (after a walks-unit source change)
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
bash "$R/scripts/profile.sh" walks 2 --tx layers9,opts5,forward2,build2,fields9
bash "$R/scripts/profile.sh" build3 2 --tx build3
bash "$R/scripts/profile.sh" optsc5 2 --tx optsc5
