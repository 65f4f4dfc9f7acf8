# LiDAR split point A/B on one box: --lidar-pipeline 3 (down blocks in the front half) vs 4 (the last down
# block in the back half beside the next batch's front), after the split-pipeline tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5
cd $R
timeout -k 10 300 python -u -m pytest tests/test_pipelines_gpu.py -x -q -m gpu -k "post_split" --timeout 200 --timeout-method thread > gpurun_out/r5/split4_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r5/split4_tests.log; exit 1; }
tail -1 gpurun_out/r5/split4_tests.log
val() { python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['lidar_pipelined'])"; }
for k in 1 2 3; do
  for m in 3 4; do
    timeout -k 10 300 python bench.py --steps 30 --warmup 5 --lidar-pipeline $m > gpurun_out/r5/split4_h_${m}_$k.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/r5/split4_h_${m}_$k.log; exit 1; }
    echo "headline --lidar-pipeline $m run $k: $(tail -1 gpurun_out/r5/split4_h_${m}_$k.log | val)"
  done
done
for m in 3 4; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --only lidar --lidar-pipeline $m > gpurun_out/r5/split4_l_${m}.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/r5/split4_l_${m}.log; exit 1; }
  echo "lidar --lidar-pipeline $m: $(tail -1 gpurun_out/r5/split4_l_${m}.log | val)"
done
