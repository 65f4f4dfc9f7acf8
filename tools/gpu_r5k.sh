# Round 5: conv_wino fp32 chain: wino + hx3 + fp32-mode + uniform tests, A/B, headline bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5
cd $R
timeout -k 10 300 python -u -m pytest tests/test_wino_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5/wino_tests.log 2>&1 || { echo WINO_TESTS_FAILED; tail -30 gpurun_out/r5/wino_tests.log; exit 1; }
tail -1 gpurun_out/r5/wino_tests.log
timeout -k 10 200 python tools/bench_wino.py > gpurun_out/r5/bench_wino.log 2>&1 || { echo BENCH_WINO_FAILED; tail -20 gpurun_out/r5/bench_wino.log; exit 1; }
cat gpurun_out/r5/bench_wino.log
timeout -k 10 600 python -u -m pytest tests/test_fp32_mode_gpu.py tests/test_bev_uniform_gpu.py tests/test_hx3_gpu.py tests/test_fast_plans.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r5/wino_fp32_tests.log 2>&1 || { echo FP32_TESTS_FAILED; tail -30 gpurun_out/r5/wino_fp32_tests.log; exit 1; }
tail -1 gpurun_out/r5/wino_fp32_tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/r5/bench_wino_headline.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/r5/bench_wino_headline.log; exit 1; }
tail -1 gpurun_out/r5/bench_wino_headline.log | cut -c1-300
