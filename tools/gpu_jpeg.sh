# JPEG ingest on MI355X: GPU tests, then bench with CompressedImage input (camera only and both branches).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_jpeg_gpu.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/jpeg_tests.log 2>&1 || { echo TESTS_FAILED; tail -40 gpurun_out/jpeg_tests.log; exit 1; }
tail -1 gpurun_out/jpeg_tests.log
timeout -k 10 300 python bench.py --camera-input jpeg --only camera --steps 30 --warmup 5 > gpurun_out/jpeg_bench_cam.log 2>&1 || { echo BENCH_CAM_FAILED; tail -20 gpurun_out/jpeg_bench_cam.log; exit 1; }
tail -1 gpurun_out/jpeg_bench_cam.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['jpeg'])"
timeout -k 10 300 python bench.py --camera-input jpeg --steps 30 --warmup 5 > gpurun_out/jpeg_bench_both.log 2>&1 || { echo BENCH_BOTH_FAILED; tail -20 gpurun_out/jpeg_bench_both.log; exit 1; }
tail -1 gpurun_out/jpeg_bench_both.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['jpeg'])"
