# Round 6: the 8-rank gloo rehearsal of bench.py (pre-flight in the JSON) and of the DP live drivers
# on one GPU, then the scalar / vector instruction mix of the LiDAR and camera steps.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
CFGS="8_local" DRIVERS=1 DRIVER_GPUS=8 bash tools/gpu_dp_rehearsal.sh || exit 1
bash tools/gpu_salu_pmc.sh
