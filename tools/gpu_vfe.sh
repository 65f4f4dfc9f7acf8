# Pillar VFE grid sizing: tests, an unpipelined LiDAR kernel trace (isolated kernel times), benches.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r4
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py tests/test_pipelines_gpu.py tests/test_pair_storage_gpu.py tests/test_bev_uniform_gpu.py > gpurun_out/r4/vfe_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -30 gpurun_out/r4/vfe_pytest.log; exit 1; }
tail -1 gpurun_out/r4/vfe_pytest.log
cd /tmp && export TMPDIR=/tmp && cd $R
rm -rf /tmp/vfe_prof
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/vfe_prof -o run -- python bench.py --only lidar --lidar-pipeline 0 --steps 8 --warmup 3 > gpurun_out/r4/vfe_prof.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/r4/vfe_prof.log; exit 1; }
f=$(find /tmp/vfe_prof -name "*kernel_trace.csv" | head -1)
python tools/step_stats.py $f --marker pc2_count --steps 6 > gpurun_out/r4/step_stats_lidar_seq_vfe.txt && grep -E "kernel time|pillar_vfe" gpurun_out/r4/step_stats_lidar_seq_vfe.txt
for rep in 1 2; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/r4/vfe_bench_$rep.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/r4/vfe_bench_$rep.log; exit 1; }
  echo "headline $rep $(tail -1 gpurun_out/r4/vfe_bench_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
