# Uniform-tile skipping in the PointPillars first block: tests, then the LiDAR-only and headline benches.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r4
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_bev_uniform_gpu.py \
  tests/test_hx3_gpu.py tests/test_pair_storage_gpu.py > gpurun_out/r4/uni_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/r4/uni_pytest.log; exit 1; }
tail -3 gpurun_out/r4/uni_pytest.log
timeout -k 10 300 python bench.py --only lidar --steps 30 --warmup 10 > gpurun_out/r4/uni_bench_lidar.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/r4/uni_bench_lidar.log; exit 1; }
tail -1 gpurun_out/r4/uni_bench_lidar.log | cut -c1-300
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/r4/uni_bench.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/r4/uni_bench.log; exit 1; }
tail -1 gpurun_out/r4/uni_bench.log | cut -c1-300
