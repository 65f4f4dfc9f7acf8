# Stem kernel: correctness tests, then a camera-only kernel trace and the headline bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r4
cd $R
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_stem_fused_gpu.py \
  tests/test_detect_fused_gpu.py tests/test_c3_fused_gpu.py > gpurun_out/r4/stem_pytest.log 2>&1 || { echo PYTEST_FAILED; tail -40 gpurun_out/r4/stem_pytest.log; exit 1; }
tail -2 gpurun_out/r4/stem_pytest.log
cd /tmp && export TMPDIR=/tmp && cd $R
rm -rf /tmp/st_prof
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/st_prof -o run -- python bench.py --only camera --steps 8 --warmup 3 > gpurun_out/r4/st_prof.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/r4/st_prof.log; exit 1; }
f=$(find /tmp/st_prof -name "*kernel_trace.csv" | head -1)
python tools/step_stats.py $f --marker yolo_stem --steps 6 > gpurun_out/r4/step_stats_camera_stem.txt && head -8 gpurun_out/r4/step_stats_camera_stem.txt
timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/r4/stem_bench.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/r4/stem_bench.log; exit 1; }
tail -1 gpurun_out/r4/stem_bench.log | cut -c1-250
