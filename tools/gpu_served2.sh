# Served path, round 2b: served GPU tests, then the served bench with the server in
# its own process — one client process pair (sliding window, shm), then P = 2 / 4
# camera + LiDAR client process pairs (the reference's one-node-per-sensor topology).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_drivers_gpu.py tests/test_detectron.py tests/test_yolov4.py tests/test_kserve.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/served_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error" gpurun_out/served_tests.log | tail -20; tail -40 gpurun_out/served_tests.log; exit 1; }
tail -1 gpurun_out/served_tests.log
timeout -k 10 300 python tools/served_bench.py --frames 512 --window 8 --server-process --wire shm --json-out gpurun_out/served2_thr_shm.json > gpurun_out/served2_thr_shm.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/served2_thr_shm.log; exit 1; }
tail -1 gpurun_out/served2_thr_shm.log | cut -c1-900
for P in 1 2 4; do
  timeout -k 10 400 python tools/served_bench.py --frames 512 --window 8 --client-procs $P --wire shm --json-out gpurun_out/served2_p${P}_shm.json > gpurun_out/served2_p${P}_shm.log 2>&1 || { echo BENCH_FAILED $P; tail -20 gpurun_out/served2_p${P}_shm.log; exit 1; }
  tail -1 gpurun_out/served2_p${P}_shm.log | cut -c1-900
done
timeout -k 10 400 python tools/served_bench.py --frames 512 --window 8 --client-procs 2 --wire raw --json-out gpurun_out/served2_p2_raw.json > gpurun_out/served2_p2_raw.log 2>&1 || { echo BENCH_FAILED raw; tail -20 gpurun_out/served2_p2_raw.log; exit 1; }
tail -1 gpurun_out/served2_p2_raw.log | cut -c1-900
