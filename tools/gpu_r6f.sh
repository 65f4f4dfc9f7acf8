# Round 6: PillarVFE walk (base: real-pillar index space, spilling at 64 VGPRs) vs the round-5 walk
# (new): same-box headline / LiDAR-only A/B plus both builds' LiDAR step kernel tables; then the VFE
# PMC passes.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
TAG=vfe RUNS=2 STATS=1 bash tools/gpu_kernels_ab.sh || exit 1
bash tools/gpu_vfe_pmc.sh
