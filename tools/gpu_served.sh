# Served path: dynamic batching + system shared memory GPU tests, then the served bench
# (server in its own process) on the raw wire and over shared memory.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
df -h /dev/shm | tail -1
timeout -k 10 400 python -u -m pytest tests/test_drivers_gpu.py -x -v -m gpu -k "served" --timeout 300 --timeout-method thread > gpurun_out/served_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error" gpurun_out/served_tests.log | tail -20; tail -40 gpurun_out/served_tests.log; exit 1; }
tail -1 gpurun_out/served_tests.log
for wire in shm raw; do
  timeout -k 10 400 python tools/served_bench.py --frames 256 --window 8 --server-process --wire $wire --json-out gpurun_out/served_proc_$wire.json > gpurun_out/served_proc_$wire.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/served_proc_$wire.log; exit 1; }
  tail -1 gpurun_out/served_proc_$wire.log | cut -c1-1000
done
