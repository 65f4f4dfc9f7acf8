# Hash-table voxeliser: order-exact GPU tests (dense / hash / auto), the SECOND-IoU and CenterPoint
# suites, and SECOND-IoU at batch 16 with the hash (auto) vs the dense grid (TCA_VOX_HASH=0).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_second.py tests/test_centerpoint.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/voxhash_tests.log 2>&1 || { echo TESTS_FAILED; grep -E 'FAILED|Error' gpurun_out/voxhash_tests.log | tail -20; tail -20 gpurun_out/voxhash_tests.log; exit 1; }
tail -1 gpurun_out/voxhash_tests.log
for m in auto 0; do
  if [ $m = auto ]; then unset TCA_VOX_HASH; else export TCA_VOX_HASH=$m; fi
  timeout -k 10 300 python bench.py --only lidar --lidar-model second_iou --batch 16 --steps 20 --warmup 5 > gpurun_out/voxhash_second_$m.log 2>&1 || { echo BENCH_FAILED $m; tail -20 gpurun_out/voxhash_second_$m.log; exit 1; }
  echo "hash=$m $(tail -1 gpurun_out/voxhash_second_$m.log | cut -c100-220)"
done
unset TCA_VOX_HASH
timeout -k 10 300 python bench.py --only lidar --steps 20 --warmup 5 > gpurun_out/voxhash_pp.log 2>&1 || { echo BENCH_FAILED pp; tail -20 gpurun_out/voxhash_pp.log; exit 1; }
echo "pointpillars $(tail -1 gpurun_out/voxhash_pp.log | cut -c100-220)"
