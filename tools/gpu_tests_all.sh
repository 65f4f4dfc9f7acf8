# The whole GPU test suite in one pytest process (stops at the first failure).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/rc3_pytest.log 2>&1 || { echo TESTS_FAILED; grep -E 'FAILED|Error' gpurun_out/rc3_pytest.log | tail -30; tail -30 gpurun_out/rc3_pytest.log; exit 1; }
tail -1 gpurun_out/rc3_pytest.log
