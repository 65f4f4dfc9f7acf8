# Round check with hx auto-selected for the wide 3x3 pair layers, then per-branch step profiles.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_round_check2.sh && TAG=${TAG:-r2_hx} bash tools/gpu_step_profile.sh
