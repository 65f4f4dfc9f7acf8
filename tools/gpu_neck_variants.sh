# fp32 neck tiling variants: GPU tests (bit identity + vs the fp64 module), then the neck micro-bench at batch 32.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_fp32_mode_gpu.py tests/test_neck.py tests/test_pair_storage_gpu.py -x -v -m gpu -k "neck or bev_plan or pipeline" --timeout 200 --timeout-method thread > gpurun_out/nv_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error" gpurun_out/nv_tests.log | tail -20; tail -30 gpurun_out/nv_tests.log; exit 1; }
tail -1 gpurun_out/nv_tests.log
timeout -k 10 300 python tools/bench_neck.py 32 1,2,3 > gpurun_out/neck_variants.json 2> gpurun_out/neck_variants.err || { echo FAILED; tail -20 gpurun_out/neck_variants.err; exit 1; }
cat gpurun_out/neck_variants.json
