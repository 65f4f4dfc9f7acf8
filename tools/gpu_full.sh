# Full GPU regression: every gpu test, headline bench, SECOND bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/full_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/full_tests.log; exit 1; }
tail -2 gpurun_out/full_tests.log
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > gpurun_out/full_bench.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/full_bench.log; exit 1; }
tail -1 gpurun_out/full_bench.log | cut -c1-260
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --batch 16 --only lidar --lidar-model second_iou > gpurun_out/full_bench_second.log 2>&1 || { echo BENCH2_FAILED; tail -30 gpurun_out/full_bench_second.log; exit 1; }
tail -1 gpurun_out/full_bench_second.log | cut -c1-260
