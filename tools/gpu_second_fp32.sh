# SECOND-IoU fp32 mode: SECOND GPU tests (sparse backbone fp32 vs fp64, f32 RoI pool, pipeline graph,
# served model), the driver families test, then the SECOND-IoU LiDAR bench at fp32 and bf16.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 500 python -u -m pytest tests/test_second.py -x -v -s -m gpu --timeout 300 --timeout-method thread > gpurun_out/sec_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|rel L2" gpurun_out/sec_tests.log | tail -20; tail -30 gpurun_out/sec_tests.log; exit 1; }
grep "rel L2" gpurun_out/sec_tests.log; tail -1 gpurun_out/sec_tests.log
for pr in fp32 bf16; do
  timeout -k 10 300 python bench.py --only lidar --lidar-model second_iou --batch 16 --steps 30 --warmup 5 --precision $pr > gpurun_out/sec_bench_$pr.log 2>&1 || { echo BENCH_FAILED $pr; tail -20 gpurun_out/sec_bench_$pr.log; exit 1; }
  tail -1 gpurun_out/sec_bench_$pr.log | cut -c1-300
done
