# Round 5 neck check: neck numerics tests, then the LiDAR-only and full benches with kernel stats.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5
cd $R
timeout -k 10 600 python -u -m pytest tests/test_neck.py tests/test_fp32_mode_gpu.py tests/test_pair_storage_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r5/neck_tests.log 2>&1 || { echo TESTS_FAILED; grep -E 'PASSED|FAILED|Error' gpurun_out/r5/neck_tests.log | tail -30; tail -40 gpurun_out/r5/neck_tests.log; exit 1; }
tail -1 gpurun_out/r5/neck_tests.log
TAG=${TAG:-r5neck} bash tools/gpu_step_profile.sh
