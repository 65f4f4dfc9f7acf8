# Non-temporal loads of the streamed point data in the LiDAR front (TCA_VOX_NT=1): the voxeliser / LiDAR
# pipeline tests with them on, then the same-box sweep (tools/gpu_knob_sweep.sh SET=15).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/r6/voxnt
TCA_VOX_NT=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
  tests/test_ops_gpu.py tests/test_pipelines_gpu.py -k "vox or lidar or pillar or pc2 or unpack" > gpurun_out/r6/voxnt/tests_nt.log 2>&1 \
  || { tail -30 gpurun_out/r6/voxnt/tests_nt.log; exit 1; }
tail -1 gpurun_out/r6/voxnt/tests_nt.log
SET=15 TAG=voxnt ROUNDS=${ROUNDS:-8} bash tools/gpu_knob_sweep.sh
