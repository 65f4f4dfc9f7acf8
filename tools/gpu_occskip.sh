# Occupancy-gated K-step skipping: pair-storage + fp32-mode + pipeline GPU tests, then the step profile.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_pair_storage_gpu.py tests/test_fp32_mode_gpu.py tests/test_pipelines_gpu.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/occ_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error" gpurun_out/occ_tests.log | tail -20; tail -30 gpurun_out/occ_tests.log; exit 1; }
tail -1 gpurun_out/occ_tests.log
TAG=r2_occskip bash tools/gpu_step_profile.sh
