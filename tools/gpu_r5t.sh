# Round 5: uniform depth with the occupancy window in LDS: tests + LiDAR-only kernel stats.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5
cd $R
timeout -k 10 300 python -u -m pytest tests/test_bev_uniform_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5/ud_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r5/ud_tests.log; exit 1; }
tail -1 gpurun_out/r5/ud_tests.log
cd /tmp && export TMPDIR=/tmp && cd $R
rm -rf /tmp/sp_ud
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/sp_ud -o run -- python bench.py --only lidar --steps 8 --warmup 3 > gpurun_out/r5/sp_ud.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/r5/sp_ud.log; exit 1; }
f=$(find /tmp/sp_ud -name "*kernel_trace.csv" | head -1)
python tools/step_stats.py $f --marker pc2_count --steps 6 > gpurun_out/r5/step_stats_lidar_ud.txt || exit 1
grep -E "step span|uniform_depth|canvas_clear" gpurun_out/r5/step_stats_lidar_ud.txt
