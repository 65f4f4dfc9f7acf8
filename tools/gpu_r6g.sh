# Round 6, LiDAR front pass 3 (new: VFE per-frame wave walk, occupancy-only canvas clear, division-free
# uniform depth / clears) vs the committed base (TCA_LAZY_CANVAS=0): exactness tests, same-box
# A/B with both builds' LiDAR step tables, then the VFE PMC passes of the new build.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
TESTS="tests/test_ops_gpu.py tests/test_fp32_mode_gpu.py tests/test_pipelines_gpu.py tests/test_centerpoint.py tests/test_bev_uniform_gpu.py tests/test_pair_storage_gpu.py" KSEL="pillar or vfe or lidar or fp32 or centerpoint or uniform or occupancy or pair" TAG=front3 RUNS=2 STATS=1 BASE_ENV=TCA_LAZY_CANVAS=0 bash tools/gpu_kernels_ab.sh || exit 1
bash tools/gpu_vfe_pmc.sh
