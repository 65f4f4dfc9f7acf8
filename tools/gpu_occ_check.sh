# Occupancy-gated first BEV conv: GPU tests (conv bit identity / garbage never read, pipeline), then the step profile.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_pair_storage_gpu.py tests/test_fp32_mode_gpu.py tests/test_pipelines_gpu.py tests/test_drivers_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/occ_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error" gpurun_out/occ_tests.log | tail -20; tail -40 gpurun_out/occ_tests.log; exit 1; }
tail -1 gpurun_out/occ_tests.log
TAG=${TAG:-r2_occ} bash tools/gpu_step_profile.sh
