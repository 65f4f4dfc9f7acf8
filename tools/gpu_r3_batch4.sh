# Round 3 batch 4: new GPU tests (DP families, captured gather plan), the live-driver bench,
# CenterPoint 1 vs 10 sweeps (LiDAR only, batch 16), headline bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_dp_gpu.py tests/test_rccl.py tests/test_centerpoint.py -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r3b4_tests.log 2>&1; echo "tests rc=$?"
grep -E "passed|failed" gpurun_out/r3b4_tests.log | tail -2; grep -E "^FAILED" gpurun_out/r3b4_tests.log | head
timeout -k 10 400 python -u tools/driver_bench.py --camera 512 --lidar 512 --batch 32 --workers 2 > gpurun_out/driver_bench.json 2> gpurun_out/driver_bench.err || { echo DRIVER_FAILED; tail -20 gpurun_out/driver_bench.err; }
cut -c1-600 gpurun_out/driver_bench.json
for sw in 1 10; do
  timeout -k 10 300 python bench.py --only lidar --lidar-model centerpoint --batch 16 --sweeps $sw --steps 20 --warmup 5 > gpurun_out/bench_cp_sweeps$sw.log 2>&1 || { echo CP_FAILED $sw; tail -20 gpurun_out/bench_cp_sweeps$sw.log; exit 1; }
  tail -1 gpurun_out/bench_cp_sweeps$sw.log | cut -c1-260
done
timeout -k 10 300 python bench.py --steps 50 --warmup 10 > gpurun_out/bench_r3_b4.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/bench_r3_b4.log; exit 1; }
tail -1 gpurun_out/bench_r3_b4.log | cut -c1-200
