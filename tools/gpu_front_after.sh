# LiDAR pipeline mode 5 with the next front gated on the first down block (TCA_FRONT_AFTER, default 1): the
# ordering tests (bit-exact against plain step()), then the same-box sweep against 0 (gpu_knob_sweep.sh SET=17).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/r6/frontafter
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_pipelines_gpu.py \
  -k "front_next or post_split" > gpurun_out/r6/frontafter/tests.log 2>&1 || { tail -30 gpurun_out/r6/frontafter/tests.log; exit 1; }
tail -1 gpurun_out/r6/frontafter/tests.log
SET=${SET:-17} TAG=frontafter${SET:-17} ROUNDS=${ROUNDS:-8} bash tools/gpu_knob_sweep.sh
