# Round 4: after 8 refinement rounds -- the 65,536-env status census again, the whole GPU suite and smoke
set -o pipefail
R=${GRAFT_REPO_ROOT:-$PWD}
cd "$R"
bash profiles/run_r04_status_census.sh || exit 1
bash profiles/run_r04l.sh
