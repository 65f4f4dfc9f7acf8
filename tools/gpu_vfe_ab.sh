# VFE kernels: tests of both variants, LiDAR-step kernel stats of each, then a same-box headline A/B
# (TCA_VFE_MFMA unset = fp32 VALU kernel, 1 = split-bf16 MFMA kernel).  Logs: gpurun_out/r5/vfe_*.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5
cd $R
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -k "pillar_vfe" tests/test_fp32_mode_gpu.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/r5/vfe_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r5/vfe_tests.log; exit 1; }
tail -1 gpurun_out/r5/vfe_tests.log
export TMPDIR=/tmp
for L in lin mfma; do
  if [ $L = mfma ]; then export TCA_VFE_MFMA=1; else unset TCA_VFE_MFMA; fi
  rm -rf /tmp/vp_$L
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/vp_$L -o run -- python bench.py --only lidar --steps 8 --warmup 3 > gpurun_out/r5/vfe_prof_$L.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/r5/vfe_prof_$L.log; exit 1; }
  f=$(find /tmp/vp_$L -name "*kernel_trace.csv" | head -1)
  python tools/step_stats.py $f --marker pc2_count --steps 6 > gpurun_out/r5/vfe_step_stats_lidar_$L.txt || exit 1
  head -8 gpurun_out/r5/vfe_step_stats_lidar_$L.txt
done
unset TCA_VFE_MFMA
VAR=TCA_VFE_MFMA A= B=1 RUNS=${RUNS:-2} TAG=vfe_h bash tools/gpu_env_ab.sh || exit 1
VAR=TCA_VFE_MFMA A= B=1 RUNS=1 TAG=vfe_l EXTRA="--only lidar" bash tools/gpu_env_ab.sh || exit 1
