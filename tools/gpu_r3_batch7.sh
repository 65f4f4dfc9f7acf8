# Round 3 batch 7: neck FM=4 variants (64 pixels per wave): bit-identity tests + timing at batch 32.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_fp32_mode_gpu.py -x -q -m gpu -k fused_neck --timeout 200 --timeout-method thread > gpurun_out/r3b7_tests.log 2>&1 || { echo TESTS_FAILED; grep -E 'FAILED|Error|assert' gpurun_out/r3b7_tests.log | head -20; tail -20 gpurun_out/r3b7_tests.log; exit 1; }
tail -1 gpurun_out/r3b7_tests.log
timeout -k 10 300 python -u tools/bench_neck.py 32 3,4,5 > gpurun_out/neck_fm4.json 2>&1 || { echo NECK_FAILED; tail -20 gpurun_out/neck_fm4.json; exit 1; }
tail -3 gpurun_out/neck_fm4.json
