# Round-4 GPU check, part 2: DP ring diagnostics, the remaining GPU tests, driver bench, layer tables.
# A step that times out, aborts or segfaults ends the script (nothing more runs on the GPU).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4
mkdir -p $O
cd $R
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2: stopping"; exit $1;; esac; }
for mode in 2d 3d; do
  echo "== dp_debug $mode"
  flag=""; [ $mode = 3d ] && flag="--three-d"
  timeout -k 10 170 python -u tools/dp_debug.py --dump 120 $flag > $O/dp_debug_$mode.log 2>&1; rc=$?
  echo "dp_debug $mode rc=$rc"
  grep -v "^\[Gloo\]" $O/dp_debug_$mode.log | tail -30
  fatal $rc dp_debug_$mode
  [ $rc -eq 0 ] || exit 1
done
echo "== tests"
timeout -k 10 1000 python -u -m pytest tests/test_dp_gpu.py tests/test_dp_drivers.py tests/test_centerpoint.py \
  tests/test_drivers_gpu.py tests/test_graph_capture_gpu.py tests/test_rccl.py \
  -v -s -m gpu --timeout 300 --timeout-method thread > $O/pytest_b.log 2>&1; rc=$?
grep -E 'PASSED|FAILED|ERROR|raw unjoined' $O/pytest_b.log | tail -60; tail -3 $O/pytest_b.log
[ $rc -eq 0 ] || { echo TESTS_RC=$rc; grep -E '^E ' $O/pytest_b.log | head -40; }
fatal $rc pytest
echo "== driver bench"
timeout -k 10 300 python -u tools/driver_bench.py --camera 1024 --lidar 1024 --batch 32 --workers 3 \
  > $O/driver_bench.json 2> $O/driver_bench.err; rc=$?
[ $rc -eq 0 ] || { echo DRIVER_BENCH_FAILED; tail -30 $O/driver_bench.err; }
fatal $rc driver_bench
cat $O/driver_bench.json
echo "== driver bench, 2 ranks on the one card (gloo rehearsal)"
TCA_DIST_BACKEND=gloo timeout -k 10 300 python -u tools/driver_bench.py --gpus 2 --camera 256 --lidar 256 --batch 32 \
  --workers 2 > $O/driver_bench_dp2.log 2>&1; rc=$?
grep -v Gloo $O/driver_bench_dp2.log | tail -5
fatal $rc driver_bench_dp2
echo "== layers"
for br in camera lidar; do
  timeout -k 10 240 python -u tools/layer_times.py --branch $br > $O/layers_$br.json 2> $O/layers_$br.txt; rc=$?
  [ $rc -eq 0 ] || { echo LAYERS_FAILED $br; tail -20 $O/layers_$br.txt; }
  fatal $rc layers_$br
  head -30 $O/layers_$br.txt
done
