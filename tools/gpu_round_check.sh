# Round check: plan-tolerance probe (prints rel L2), smoke(), the whole GPU suite, the default bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_fast_plans.py -x -v -s -m gpu --timeout 200 --timeout-method thread > gpurun_out/rc2_plans.log 2>&1 || { echo PLANS_FAILED; tail -30 gpurun_out/rc2_plans.log; exit 1; }
grep "rel L2" gpurun_out/rc2_plans.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/rc2_smoke.log 2>&1 || { echo SMOKE_FAILED; tail -30 gpurun_out/rc2_smoke.log; exit 1; }
tail -1 gpurun_out/rc2_smoke.log
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/rc2_pytest.log 2>&1 || { echo TESTS_FAILED; grep -E 'FAILED|Error' gpurun_out/rc2_pytest.log | tail -30; tail -30 gpurun_out/rc2_pytest.log; exit 1; }
tail -1 gpurun_out/rc2_pytest.log
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/rc2_bench.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/rc2_bench.log; exit 1; }
tail -1 gpurun_out/rc2_bench.log | cut -c1-300
