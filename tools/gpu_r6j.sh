# Round 6: the final kernels against the round-start (round-5 final) build on one box:
# headline + LiDAR-only, 3 rounds alternating, and both builds' LiDAR step tables.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p triton_client_amd/_lib/ab
cp triton_client_amd/_lib/ab/libtca_kernels_r5.so triton_client_amd/_lib/ab/libtca_kernels_base.so
TAG=r6vsr5 RUNS=3 STATS=1 BASE_ENV=TCA_LAZY_CANVAS=0 bash tools/gpu_kernels_ab.sh
