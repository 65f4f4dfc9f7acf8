# Sparse-gather stride-2 conv (conv_s2sp.hip): its tests and the plan / pipeline tests, LiDAR-step
# kernel stats with it on and off, then a same-box headline A/B (TCA_S2SP unset = on, 0 = dense hx3s2).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5
cd $R
timeout -k 10 400 python -u -m pytest tests/test_hx3_gpu.py tests/test_pair_storage_gpu.py tests/test_fast_plans.py tests/test_fp32_mode_gpu.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/r5/s2sp_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/r5/s2sp_tests.log | head -20; tail -30 gpurun_out/r5/s2sp_tests.log; exit 1; }
tail -1 gpurun_out/r5/s2sp_tests.log
export TMPDIR=/tmp
for L in on off; do
  if [ $L = off ]; then export TCA_S2SP=0; else unset TCA_S2SP; fi
  rm -rf /tmp/sp_$L
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/sp_$L -o run -- python bench.py --only lidar --steps 8 --warmup 3 > gpurun_out/r5/s2sp_prof_$L.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/r5/s2sp_prof_$L.log; exit 1; }
  f=$(find /tmp/sp_$L -name "*kernel_trace.csv" | head -1)
  python tools/step_stats.py $f --marker pc2_count --steps 6 > gpurun_out/r5/s2sp_step_stats_lidar_$L.txt || exit 1
  head -12 gpurun_out/r5/s2sp_step_stats_lidar_$L.txt
done
unset TCA_S2SP
VAR=TCA_S2SP A= B=0 RUNS=${RUNS:-2} TAG=s2sp_h bash tools/gpu_env_ab.sh || exit 1
VAR=TCA_S2SP A= B=0 RUNS=1 TAG=s2sp_l EXTRA="--only lidar" bash tools/gpu_env_ab.sh || exit 1
VAR=TCA_S2SP_TILE A= B=1 RUNS=2 TAG=s2sp_tile_l EXTRA="--only lidar" bash tools/gpu_env_ab.sh || exit 1
