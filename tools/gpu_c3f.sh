# Fused C3 kernels (c3_fused.hip): numerics vs the unfused chain, camera fp32 gates, per-layer
# table and camera-only bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4
mkdir -p $O
cd $R
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2: stopping"; exit $1;; esac; }
timeout -k 10 600 python -u -m pytest tests/test_c3_fused_gpu.py tests/test_stem_fused_gpu.py tests/test_fp32_mode_gpu.py \
  -v -m gpu --timeout 300 --timeout-method thread -k "c3 or camera or yolo or headline" > $O/pytest_c3f.log 2>&1; rc=$?
grep -E 'PASSED|FAILED|ERROR' $O/pytest_c3f.log | tail -40; tail -2 $O/pytest_c3f.log
[ $rc -eq 0 ] || { echo TESTS_RC=$rc; grep -E '^E ' $O/pytest_c3f.log | head -30; }
fatal $rc pytest
timeout -k 10 240 python -u tools/layer_times.py --branch camera > $O/layers_camera_c3f.json 2> $O/layers_camera_c3f.txt; rc=$?
fatal $rc layers
head -25 $O/layers_camera_c3f.txt
timeout -k 10 300 python -u bench.py --only camera --steps 30 --warmup 5 > $O/bench_camera_c3f.json 2> $O/bench_camera_c3f.err; rc=$?
fatal $rc bench_cam
cut -c1-300 $O/bench_camera_c3f.json
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 > $O/bench_c3f.json 2> $O/bench_c3f.err; rc=$?
fatal $rc bench
cut -c1-300 $O/bench_c3f.json
