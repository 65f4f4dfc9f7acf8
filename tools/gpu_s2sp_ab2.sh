# conv_s2sp tiles: tests, LiDAR-step kernel stats (default), LiDAR-only runs for dense / 4 x 32 / 2 x 32
# alternating, then the headline with the default against the dense kernel.  Logs: gpurun_out/r5/s2sp2_*.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5
cd $R
timeout -k 10 400 python -u -m pytest tests/test_hx3_gpu.py tests/test_pair_storage_gpu.py -x -v -m gpu -k "s2sp or occupancy" --timeout 200 --timeout-method thread > gpurun_out/r5/s2sp2_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/r5/s2sp2_tests.log | head -20; exit 1; }
tail -1 gpurun_out/r5/s2sp2_tests.log
export TMPDIR=/tmp
rm -rf /tmp/sp2
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/sp2 -o run -- python bench.py --only lidar --steps 8 --warmup 3 > gpurun_out/r5/s2sp2_prof.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/r5/s2sp2_prof.log; exit 1; }
f=$(find /tmp/sp2 -name "*kernel_trace.csv" | head -1)
python tools/step_stats.py $f --marker pc2_count --steps 6 > gpurun_out/r5/s2sp2_step_stats_lidar.txt || exit 1
head -12 gpurun_out/r5/s2sp2_step_stats_lidar.txt
val() { python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"; }
for k in 1 2; do
  for cfg in "TCA_S2SP=0" "TCA_S2SP_TILE=0" "TCA_S2SP_TILE=2"; do
    env $cfg timeout -k 10 300 python bench.py --only lidar --steps 30 --warmup 5 > gpurun_out/r5/s2sp2_l_${cfg}_$k.log 2>&1 || { echo BENCH_FAILED; tail -5 gpurun_out/r5/s2sp2_l_${cfg}_$k.log; exit 1; }
    echo "lidar $cfg run $k: $(tail -1 gpurun_out/r5/s2sp2_l_${cfg}_$k.log | val)"
  done
done
VAR=TCA_S2SP A= B=0 RUNS=2 TAG=s2sp2_h bash tools/gpu_env_ab.sh || exit 1
