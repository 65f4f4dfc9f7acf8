# Pipelined step: canvas clear + voxeliser reset on a side stream after the first conv
# (TCA_LIDAR_SIDE_CLEAN=1, default) vs in line; GPU pipeline tests first.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_pipelines_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/sc_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/sc_tests.log; exit 1; }
tail -1 gpurun_out/sc_tests.log
for k in 1 2; do
for v in 1 0; do
  TCA_LIDAR_SIDE_CLEAN=$v timeout -k 10 300 python bench.py --steps 50 --warmup 10 > gpurun_out/sc_$v.log 2>&1 || { echo BENCH_FAILED $v; tail -30 gpurun_out/sc_$v.log; exit 1; }
  echo "side_clean=$v $(tail -1 gpurun_out/sc_$v.log | cut -c100-200) 3d=$(grep -o '"avg_3d_dets_per_frame": [0-9.]*' gpurun_out/sc_$v.log) 2d=$(grep -o '"avg_2d_dets_per_frame": [0-9.]*' gpurun_out/sc_$v.log)"
done
done
