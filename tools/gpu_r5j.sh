# Round 5: conv_wino.hip iteration: tests + A/B against hx3 only.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5
cd $R
timeout -k 10 300 python -u -m pytest tests/test_wino_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5/wino_tests.log 2>&1 || { echo WINO_TESTS_FAILED; tail -30 gpurun_out/r5/wino_tests.log; exit 1; }
tail -1 gpurun_out/r5/wino_tests.log
timeout -k 10 200 python tools/bench_wino.py > gpurun_out/r5/bench_wino.log 2>&1 || { echo BENCH_WINO_FAILED; tail -20 gpurun_out/r5/bench_wino.log; exit 1; }
cat gpurun_out/r5/bench_wino.log
