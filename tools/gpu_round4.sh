# Round-4 GPU check: live-driver + DP ring GPU tests, then the driver bench.
#   usage: bash tools/gpu_round4.sh
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests/test_draw.py tests/test_live.py tests/test_dp_gpu.py tests/test_dp_drivers.py \
  tests/test_centerpoint.py tests/test_drivers_gpu.py tests/test_graph_capture_gpu.py tests/test_rccl.py -v -m gpu --timeout 300 --timeout-method thread \
  > $O/pytest.log 2>&1; rc=$?
grep -E 'PASSED|FAILED|ERROR' $O/pytest.log | tail -60; tail -3 $O/pytest.log
[ $rc -eq 0 ] || { echo TESTS_RC=$rc; grep -E '^E ' $O/pytest.log | head -40; }
timeout -k 10 300 python -u tools/driver_bench.py --camera 1024 --lidar 1024 --batch 32 --workers 3 \
  > $O/driver_bench.json 2> $O/driver_bench.err || { echo DRIVER_BENCH_FAILED; tail -30 $O/driver_bench.err; exit 1; }
cat $O/driver_bench.json
for br in camera lidar; do
  timeout -k 10 240 python -u tools/layer_times.py --branch $br > $O/layers_$br.json 2> $O/layers_$br.txt || { echo LAYERS_FAILED $br; tail -20 $O/layers_$br.txt; exit 1; }
  head -25 $O/layers_$br.txt
done
