# fp32 precision mode: kernel + end-to-end parity tests, existing GPU suites, fp32 and bf16 bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_fp32_mode_gpu.py -x -v -s -m gpu --timeout 300 --timeout-method thread > gpurun_out/fp32_tests.log 2>&1 || { echo FP32_TESTS_FAILED; tail -40 gpurun_out/fp32_tests.log; exit 1; }
tail -3 gpurun_out/fp32_tests.log
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_fp32.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/bench_fp32.log; exit 1; }
tail -1 gpurun_out/bench_fp32.log | cut -c1-300
