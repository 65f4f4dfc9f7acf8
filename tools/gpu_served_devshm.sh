# Device shared memory round 3: served tests, devshm at GIL switch 2e-4 / 5e-5, shm, raw.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_drivers_gpu.py -x -q -m gpu -k "shared_memory or dynamic_batch" --timeout 300 --timeout-method thread > gpurun_out/devshm3_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|error" gpurun_out/devshm3_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/devshm3_tests.log
NOTEST=1 WIRES="devshm" bash tools/gpu_served3.sh || exit 1
mv gpurun_out/served3_prof_p4_s1_devshm.json gpurun_out/served3_prof_p4_s1_devshm_sw2e4.json
TCA_GIL_SWITCH_S=5e-5 NOTEST=1 WIRES="devshm shm raw" bash tools/gpu_served3.sh
