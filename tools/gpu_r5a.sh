# Round 5: remote-client device path tests, NUMA on the box, rank-0 fan-out copy rate.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5
cd $R
timeout -k 10 600 python -u -m pytest tests/test_remote_device_gpu.py tests/test_numa_gpu.py tests/test_live.py tests/test_graph_capture_gpu.py -x -v -s -m gpu --timeout 300 --timeout-method thread > gpurun_out/r5/remote_tests.log 2>&1 || { echo TESTS_FAILED; grep -E 'PASSED|FAILED|Error' gpurun_out/r5/remote_tests.log | tail -30; tail -40 gpurun_out/r5/remote_tests.log; exit 1; }
grep -E 'PASSED|passed|failed' gpurun_out/r5/remote_tests.log | tail -12
grep '"info"' gpurun_out/r5/remote_tests.log | head -1
timeout -k 10 300 python tools/fanout_bench.py --threads 4,8,16,32 --json gpurun_out/r5/fanout.json > gpurun_out/r5/fanout.log 2>&1 || { echo FANOUT_FAILED; tail -20 gpurun_out/r5/fanout.log; exit 1; }
cat gpurun_out/r5/fanout.log
MARKER=pc2_count bash tools/gpu_timeline.sh > gpurun_out/r5/timeline.txt 2>&1 || { echo TIMELINE_FAILED; tail -20 gpurun_out/r5/timeline.txt; exit 1; }
cp gpurun_out/tl_full_steps.txt gpurun_out/r5/tl_full_steps_base.txt
head -2 gpurun_out/r5/tl_full_steps_base.txt
