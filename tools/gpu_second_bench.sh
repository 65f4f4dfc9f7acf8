set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_second.py tests/test_ops_gpu.py tests/test_pipelines_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/second_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/second_tests.log; exit 1; }
tail -2 gpurun_out/second_tests.log
timeout -k 10 300 python tools/second_probe.py > gpurun_out/second_probe.log 2>&1 || { echo PROBE_FAILED; tail -40 gpurun_out/second_probe.log; exit 1; }
cat gpurun_out/second_probe.log
