set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5
cd /tmp && export TMPDIR=/tmp && cd $R
for L in new base; do
  if [ $L = base ]; then export TCA_KERNELS_LIB=$R/triton_client_amd/_lib/ab/libtca_kernels_base.so; else unset TCA_KERNELS_LIB; fi
  rm -rf /tmp/vp_$L
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/vp_$L -o run -- python bench.py --only lidar --steps 8 --warmup 3 > gpurun_out/r5/vp_$L.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/r5/vp_$L.log; exit 1; }
  f=$(find /tmp/vp_$L -name "*kernel_trace.csv" | head -1)
  python tools/step_stats.py $f --marker pc2_count --steps 6 > gpurun_out/r5/step_stats_lidar_vfe64_$L.txt || exit 1
  head -8 gpurun_out/r5/step_stats_lidar_vfe64_$L.txt
done
