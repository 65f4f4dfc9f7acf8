# Round 6, LiDAR front pass 3 (new: VFE per-frame wave walk, occupancy-only canvas clear, division-free
# uniform depth / clears) vs the committed base (TCA_LAZY_CANVAS=0): same-box A/B with both builds'
# LiDAR step tables, then the VFE PMC passes of the new build.  (The exactness tests of this pass:
# TESTS=... below; 210 passed on the box, profiles/r6/front3/.)
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
TESTS="$T3" KSEL="pillar or vfe or lidar or fp32 or centerpoint or uniform or occupancy or pair" TAG=front3 RUNS=2 STATS=1 BASE_ENV=TCA_LAZY_CANVAS=0 bash tools/gpu_kernels_ab.sh || exit 1
bash tools/gpu_vfe_pmc.sh
