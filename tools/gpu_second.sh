set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_second.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/second_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/second_tests.log; exit 1; }
tail -5 gpurun_out/second_tests.log
