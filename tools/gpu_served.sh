# Served path on MI355X: served-vs-local GPU test, then the served-path bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_drivers_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/served_tests.log 2>&1 || { echo TESTS_FAILED; grep -E 'PASSED|FAILED|Error' gpurun_out/served_tests.log | tail -20; tail -30 gpurun_out/served_tests.log; exit 1; }
tail -1 gpurun_out/served_tests.log
timeout -k 10 400 python tools/served_bench.py --frames ${FRAMES:-96} --window ${WINDOW:-8} --json-out gpurun_out/served_bench.json > gpurun_out/served_bench.log 2>&1 || { echo SERVED_BENCH_FAILED; tail -20 gpurun_out/served_bench.log; exit 1; }
tail -1 gpurun_out/served_bench.log
