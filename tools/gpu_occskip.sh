# hx3s2 empty-tile skip: stride-2 / occupancy GPU tests, then the LiDAR-only and headline benches.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_hx3_gpu.py tests/test_pair_storage_gpu.py tests/test_fp32_mode_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/occskip_tests.log 2>&1 || { echo TESTS_FAILED; grep -E 'FAILED|Error' gpurun_out/occskip_tests.log | tail -20; exit 1; }
tail -1 gpurun_out/occskip_tests.log
for k in 1 2; do
  timeout -k 10 300 python bench.py --only lidar --steps 30 --warmup 5 > gpurun_out/occskip_lidar_$k.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/occskip_lidar_$k.log; exit 1; }
  echo "lidar $(tail -1 gpurun_out/occskip_lidar_$k.log | cut -c100-200)"
done
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > gpurun_out/occskip_both.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/occskip_both.log; exit 1; }
echo "both $(tail -1 gpurun_out/occskip_both.log | cut -c100-200)"
cd /tmp && export TMPDIR=/tmp && cd $R
rm -rf /tmp/occsk
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/occsk -o run -- python bench.py --only lidar --steps 8 --warmup 3 > gpurun_out/occskip_prof.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/occskip_prof.log; exit 1; }
f=$(find /tmp/occsk -name "*kernel_trace.csv" | head -1)
python tools/step_stats.py $f --marker pc2_count --steps 6 > gpurun_out/step_stats_lidar_occskip.txt || exit 1
head -12 gpurun_out/step_stats_lidar_occskip.txt
