# Run the given GPU test files (or all GPU tests), one pytest process, then optionally the default bench.
#   usage: bash tools/gpu_pytest.sh [test paths...]   env BENCH=1 adds `python bench.py --steps 20 --warmup 5`
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
T=${*:-tests}
timeout -k 10 1000 python -u -m pytest $T -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest.log 2>&1 || { echo TESTS_FAILED; grep -E 'PASSED|FAILED|Error|error' gpurun_out/pytest.log | tail -30; tail -30 gpurun_out/pytest.log; exit 1; }
grep -cE 'PASSED' gpurun_out/pytest.log; tail -1 gpurun_out/pytest.log
if [ -n "$BENCH" ]; then
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/bench.log; exit 1; }
  tail -1 gpurun_out/bench.log | cut -c1-400
fi
