# Fused YOLOv5 Detect + filter: tests, then camera-only and headline benches (A/B via DETECT_FUSED).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r4
cd $R
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_detect_fused_gpu.py \
  tests/test_c3_fused_gpu.py tests/test_pipelines_gpu.py > gpurun_out/r4/det_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/r4/det_pytest.log; exit 1; }
tail -3 gpurun_out/r4/det_pytest.log
timeout -k 10 300 python bench.py --only camera --steps 30 --warmup 10 > gpurun_out/r4/det_bench_camera.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/r4/det_bench_camera.log; exit 1; }
tail -1 gpurun_out/r4/det_bench_camera.log | cut -c1-250
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/r4/det_bench.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/r4/det_bench.log; exit 1; }
tail -1 gpurun_out/r4/det_bench.log | cut -c1-250
cd /tmp && export TMPDIR=/tmp && cd $R
rm -rf /tmp/det_prof
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/det_prof -o run -- python bench.py --only camera --steps 8 --warmup 3 > gpurun_out/r4/det_prof.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/r4/det_prof.log; exit 1; }
f=$(find /tmp/det_prof -name "*kernel_trace.csv" | head -1)
python tools/step_stats.py $f --marker yolo_stem --steps 6 > gpurun_out/r4/step_stats_camera_det.txt && head -14 gpurun_out/r4/step_stats_camera_det.txt
