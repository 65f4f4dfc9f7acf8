# Device shared memory (HIP IPC) served path: GPU test, then the served bench over devshm / shm.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
echo "IPC legacy mode: ${HSA_ENABLE_IPC_MODE_LEGACY:-unset}"
timeout -k 10 400 python -u -m pytest tests/test_drivers_gpu.py -x -v -m gpu -k "device_shared_memory or shared_memory_matches" --timeout 300 --timeout-method thread > gpurun_out/devshm_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|error" gpurun_out/devshm_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/devshm_tests.log
NOTEST=1 WIRES="devshm shm" bash tools/gpu_served3.sh
