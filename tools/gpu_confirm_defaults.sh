# Round 6: the new defaults (neck tiling 2, two-pillar VFE): their tests, a same-box sweep against the round-start
# defaults (tools/gpu_knob_sweep.sh SET=3), then the driver's command three times.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/r6/confirm
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_fp32_mode_gpu.py tests/test_pipelines_gpu.py -x -q -m gpu -k "vfe or neck or lidar or pillar" --timeout 200 --timeout-method thread > gpurun_out/r6/confirm/tests.log 2>&1 || { echo TESTS_FAILED; tail -20 gpurun_out/r6/confirm/tests.log; exit 1; }
tail -1 gpurun_out/r6/confirm/tests.log
SET=3 ROUNDS=5 TAG=knobs3 bash tools/gpu_knob_sweep.sh || exit 1
for k in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r6/confirm/driver_$k.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/r6/confirm/driver_$k.log; exit 1; }
  echo "driver-style $k $(tail -1 gpurun_out/r6/confirm/driver_$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done
