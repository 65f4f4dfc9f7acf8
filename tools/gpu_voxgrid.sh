# Bounded-grid per-point voxeliser passes: exactness with a tiny grid (many chunks per workgroup) and
# the default, then the same-box sweep (tools/gpu_knob_sweep.sh SET=13).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/r6/voxgrid
TCA_VOX_GRID=3 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_ops_gpu.py tests/test_pipelines_gpu.py -k "vox or lidar or pillar" > gpurun_out/r6/voxgrid/tests_g3.log 2>&1 \
  || { tail -30 gpurun_out/r6/voxgrid/tests_g3.log; exit 1; }
tail -2 gpurun_out/r6/voxgrid/tests_g3.log
SET=13 TAG=voxgrid ROUNDS=${ROUNDS:-3} bash tools/gpu_knob_sweep.sh
