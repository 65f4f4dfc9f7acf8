# YOLOv4 fp32 mode: YOLOv4 GPU tests (plan vs fp64 in both precisions, pipeline graph, served model),
# then the camera-only YOLOv4 bench at fp32 and bf16.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_yolov4.py -x -v -s -m gpu --timeout 300 --timeout-method thread > gpurun_out/y4_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|rel L2" gpurun_out/y4_tests.log | tail -20; tail -30 gpurun_out/y4_tests.log; exit 1; }
grep "rel L2" gpurun_out/y4_tests.log; tail -1 gpurun_out/y4_tests.log
for pr in fp32 bf16; do
  timeout -k 10 300 python bench.py --only camera --camera-model yolov4 --batch 16 --steps 30 --warmup 5 --precision $pr > gpurun_out/y4_bench_$pr.log 2>&1 || { echo BENCH_FAILED $pr; tail -20 gpurun_out/y4_bench_$pr.log; exit 1; }
  tail -1 gpurun_out/y4_bench_$pr.log | cut -c1-300
done
