# Round-end style check: smoke(), the full GPU test suite, the default bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/rc_smoke.log 2>&1 || { echo SMOKE_FAILED; tail -30 gpurun_out/rc_smoke.log; exit 1; }
tail -1 gpurun_out/rc_smoke.log
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/rc_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/rc_tests.log; exit 1; }
tail -1 gpurun_out/rc_tests.log
timeout -k 10 300 python bench.py > gpurun_out/rc_bench.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/rc_bench.log; exit 1; }
tail -1 gpurun_out/rc_bench.log | cut -c1-200
