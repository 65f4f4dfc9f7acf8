# Round 6: --lidar-pipeline 5 (the LiDAR front leaves the critical stream): its ordering test, then a same-box
# sweep against the default mode 3 (tools/gpu_knob_sweep.sh SET=5).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/r6/pipe5
timeout -k 10 400 python -u -m pytest tests/test_pipelines_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r6/pipe5/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r6/pipe5/tests.log; exit 1; }
tail -1 gpurun_out/r6/pipe5/tests.log
SET=5 ROUNDS=${ROUNDS:-4} TAG=knobs5 bash tools/gpu_knob_sweep.sh
