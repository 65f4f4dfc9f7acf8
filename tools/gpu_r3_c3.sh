# Merged C3 cv1|cv2: plan numerics tests, then the headline bench + per-branch step tables.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 500 python -u -m pytest tests/test_fast_plans.py tests/test_fp32_mode_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/c3_tests.log 2>&1 || { echo TESTS_FAILED; grep -E 'FAILED|Error|assert' gpurun_out/c3_tests.log | head -20; tail -20 gpurun_out/c3_tests.log; exit 1; }
tail -1 gpurun_out/c3_tests.log
TAG=r3_c3 bash tools/gpu_step_profile.sh
