# Round-4 GPU check, part 2: DP ring diagnostics, the remaining GPU tests, driver bench, layer tables.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4
mkdir -p $O
cd $R
echo "== dp_debug 2d"
timeout -k 10 170 python -u tools/dp_debug.py --dump 100 > $O/dp_debug_2d.log 2>&1; echo "dp_debug rc=$?"
grep -v "^\[Gloo\]" $O/dp_debug_2d.log | tail -40
echo "== tests"
timeout -k 10 900 python -u -m pytest tests/test_centerpoint.py tests/test_drivers_gpu.py tests/test_graph_capture_gpu.py \
  tests/test_rccl.py -v -s -m gpu --timeout 300 --timeout-method thread > $O/pytest_b.log 2>&1; rc=$?
grep -E 'PASSED|FAILED|ERROR|raw unjoined' $O/pytest_b.log | tail -60; tail -3 $O/pytest_b.log
[ $rc -eq 0 ] || { echo TESTS_RC=$rc; grep -E '^E ' $O/pytest_b.log | head -40; }
echo "== driver bench"
timeout -k 10 300 python -u tools/driver_bench.py --camera 1024 --lidar 1024 --batch 32 --workers 3 \
  > $O/driver_bench.json 2> $O/driver_bench.err || { echo DRIVER_BENCH_FAILED; tail -30 $O/driver_bench.err; }
cat $O/driver_bench.json
echo "== layers"
for br in camera lidar; do
  timeout -k 10 240 python -u tools/layer_times.py --branch $br > $O/layers_$br.json 2> $O/layers_$br.txt || { echo LAYERS_FAILED $br; tail -20 $O/layers_$br.txt; }
  head -30 $O/layers_$br.txt
done
