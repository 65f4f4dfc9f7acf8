# Device shared memory round 2: copy kernel + served tests, then devshm at 1 / 2 server processes, shm.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_drivers_gpu.py -x -q -m gpu -k "copy_segments or shared_memory or dynamic_batch or batch_plans" --timeout 300 --timeout-method thread > gpurun_out/devshm2_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|error" gpurun_out/devshm2_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/devshm2_tests.log
NOTEST=1 WIRES="devshm shm" bash tools/gpu_served3.sh || exit 1
SPROCS=2 NOTEST=1 WIRES="devshm" bash tools/gpu_served3.sh
