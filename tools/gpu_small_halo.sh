# Small-halo conv (tile 60) numerics, then the round-end check and a camera-only bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -v -m gpu -k "small_halo or fused_conv" --timeout 120 --timeout-method thread > gpurun_out/small_halo_tests.log 2>&1 || { echo SH_TESTS_FAILED; tail -40 gpurun_out/small_halo_tests.log; exit 1; }
tail -1 gpurun_out/small_halo_tests.log
timeout -k 10 200 python bench.py --only camera --steps 100 --warmup 10 > gpurun_out/small_halo_cam.log 2>&1 || { echo CAM_FAILED; tail -30 gpurun_out/small_halo_cam.log; exit 1; }
tail -1 gpurun_out/small_halo_cam.log | cut -c1-300
bash tools/gpu_round_check.sh
