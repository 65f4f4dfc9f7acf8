# Halo conv (tile 50) regression: conv numerics, LiDAR pipeline tests, conv timing, headline bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py tests/test_pipelines_gpu.py -x -q -m gpu -k "conv or lidar or centerpoint or halo" --timeout 120 --timeout-method thread > gpurun_out/halo_check_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/halo_check_tests.log; exit 1; }
tail -1 gpurun_out/halo_check_tests.log
timeout -k 10 120 python tools/bench_conv.py 22,41,50 pp.b1.conv > gpurun_out/halo_conv.log 2>&1 || { echo CONV_FAILED; tail -5 gpurun_out/halo_conv.log; exit 1; }
grep "^{" gpurun_out/halo_conv.log
for i in 1 2; do timeout -k 10 200 python bench.py --steps 50 --warmup 5 > gpurun_out/halo_bench_$i.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/halo_bench_$i.log; exit 1; }; tail -1 gpurun_out/halo_bench_$i.log | cut -c100-200; done
timeout -k 10 200 python bench.py --steps 100 --warmup 10 --only lidar > gpurun_out/halo_bench_lidar.log 2>&1 && tail -1 gpurun_out/halo_bench_lidar.log | cut -c100-200
