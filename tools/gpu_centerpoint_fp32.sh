# CenterPoint fp32 mode: CenterPoint GPU tests (PFN / plan vs fp64, pipeline fp32 vs bf16, graph), the
# served / local 3D family tests, then the CenterPoint LiDAR bench at fp32 and bf16.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 500 python -u -m pytest tests/test_centerpoint.py tests/test_drivers_gpu.py -x -v -s -m gpu --timeout 300 --timeout-method thread > gpurun_out/cp_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|rel L2" gpurun_out/cp_tests.log | tail -20; tail -30 gpurun_out/cp_tests.log; exit 1; }
grep "rel L2" gpurun_out/cp_tests.log; tail -1 gpurun_out/cp_tests.log
for pr in fp32 bf16; do
  timeout -k 10 300 python bench.py --only lidar --lidar-model centerpoint --batch 16 --steps 30 --warmup 5 --precision $pr > gpurun_out/cp_bench_$pr.log 2>&1 || { echo BENCH_FAILED $pr; tail -20 gpurun_out/cp_bench_$pr.log; exit 1; }
  tail -1 gpurun_out/cp_bench_$pr.log | cut -c1-400
done
