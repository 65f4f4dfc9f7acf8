# New-feature GPU check: native RCCL communicator + LiDAR-family local engines, then the full suite + headline bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_rccl.py tests/test_drivers_gpu.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/new_tests.log 2>&1 || { echo NEW_TESTS_FAILED; tail -40 gpurun_out/new_tests.log; exit 1; }
tail -3 gpurun_out/new_tests.log
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/full_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/full_tests.log; exit 1; }
tail -2 gpurun_out/full_tests.log
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > gpurun_out/full_bench.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/full_bench.log; exit 1; }
tail -1 gpurun_out/full_bench.log | cut -c1-300
