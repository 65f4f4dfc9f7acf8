# Served path with server-side dynamic batching: GPU tests, then the served bench (in-process and
# server-process topologies).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_drivers_gpu.py -x -v -m gpu -k "served" --timeout 300 --timeout-method thread > gpurun_out/served_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error" gpurun_out/served_tests.log | tail -20; tail -40 gpurun_out/served_tests.log; exit 1; }
tail -1 gpurun_out/served_tests.log
for w in 8 16; do
  timeout -k 10 400 python tools/served_bench.py --frames 256 --window $w --server-process --json-out gpurun_out/served_proc_w$w.json > gpurun_out/served_proc_w$w.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/served_proc_w$w.log; exit 1; }
  tail -1 gpurun_out/served_proc_w$w.log | cut -c1-900
done
