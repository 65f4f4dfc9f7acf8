# Sparse-gather stride-2 conv (conv_s2sp.hip, opt-in TCA_S2SP=1) against the default dense hx3s2 kernel:
# its tests and the occupancy pipeline tests, LiDAR-step kernel stats of both, LiDAR-only runs of the dense
# kernel and the 4 x 32 / 2 x 32 / 8 x 32 tiles alternating, then the headline on / off.  Logs: gpurun_out/r5/s2sp_*.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5
cd $R
timeout -k 10 400 python -u -m pytest tests/test_hx3_gpu.py tests/test_pair_storage_gpu.py -x -v -m gpu -k "s2sp or occupancy" --timeout 200 --timeout-method thread > gpurun_out/r5/s2sp_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/r5/s2sp_tests.log | head -20; exit 1; }
tail -1 gpurun_out/r5/s2sp_tests.log
export TMPDIR=/tmp
for L in on off; do
  if [ $L = on ]; then export TCA_S2SP=1; else unset TCA_S2SP; fi
  rm -rf /tmp/sp_$L
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/sp_$L -o run -- python bench.py --only lidar --steps 8 --warmup 3 > gpurun_out/r5/s2sp_prof_$L.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/r5/s2sp_prof_$L.log; exit 1; }
  f=$(find /tmp/sp_$L -name "*kernel_trace.csv" | head -1)
  python tools/step_stats.py $f --marker pc2_count --steps 6 > gpurun_out/r5/s2sp_step_stats_lidar_$L.txt || exit 1
  head -12 gpurun_out/r5/s2sp_step_stats_lidar_$L.txt
done
unset TCA_S2SP
val() { python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"; }
for k in 1 2; do
  for cfg in "TCA_S2SP=0" "TCA_S2SP=1" "TCA_S2SP_TILE=2 TCA_S2SP=1" "TCA_S2SP_TILE=1 TCA_S2SP=1"; do
    tag=$(echo $cfg | tr ' =' '__')
    env $cfg timeout -k 10 300 python bench.py --only lidar --steps 30 --warmup 5 > gpurun_out/r5/s2sp_l_${tag}_$k.log 2>&1 || { echo BENCH_FAILED; tail -5 gpurun_out/r5/s2sp_l_${tag}_$k.log; exit 1; }
    echo "lidar $cfg run $k: $(tail -1 gpurun_out/r5/s2sp_l_${tag}_$k.log | val)"
  done
done
VAR=TCA_S2SP A= B=1 RUNS=2 TAG=s2sp_h bash tools/gpu_env_ab.sh || exit 1
