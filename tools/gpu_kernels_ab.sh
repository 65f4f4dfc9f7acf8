# Round 5: VFE three-deep load pipeline A/B (TCA_KERNELS_LIB = the previous build): VFE tests, LiDAR-only
# and headline, two runs each, same box.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5
cd $R
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_pipelines_gpu.py -x -q -m gpu -k "pillar or vfe or lidar" --timeout 200 --timeout-method thread > gpurun_out/r5/vfe3_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r5/vfe3_tests.log; exit 1; }
tail -1 gpurun_out/r5/vfe3_tests.log
BASE=$R/triton_client_amd/_lib/ab/libtca_kernels_base.so
for k in 1 2; do
  for L in new base; do
    if [ $L = base ]; then export TCA_KERNELS_LIB=$BASE; else unset TCA_KERNELS_LIB; fi
    timeout -k 10 300 python bench.py --only lidar --steps 30 --warmup 5 > gpurun_out/r5/vfe3_l_${L}_$k.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/r5/vfe3_l_${L}_$k.log; exit 1; }
    timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/r5/vfe3_h_${L}_$k.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/r5/vfe3_h_${L}_$k.log; exit 1; }
    echo "$L run $k: lidar $(tail -1 gpurun_out/r5/vfe3_l_${L}_$k.log | cut -c100-130) headline $(tail -1 gpurun_out/r5/vfe3_h_${L}_$k.log | cut -c100-130)"
  done
done
