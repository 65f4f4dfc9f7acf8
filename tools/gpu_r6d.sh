# Round 6: the LiDAR front, second pass (bounded-grid canvas clear / slot reset, coalesced voxel-count
# scan, VFE walking only real pillars): exactness tests, same-box A/B against the saved base build,
# LiDAR step kernel stats.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6
cd $R
TESTS="tests/test_ops_gpu.py tests/test_fp32_mode_gpu.py tests/test_pipelines_gpu.py tests/test_centerpoint.py tests/test_second.py" KSEL="voxel or pc2 or lidar or pillar or fp32 or vfe or centerpoint or second" TAG=front2 RUNS=2 bash tools/gpu_kernels_ab.sh || exit 1
cd /tmp && export TMPDIR=/tmp && cd $R
rm -rf /tmp/sp_lidar
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/sp_lidar -o run -- python bench.py --only lidar --steps 8 --warmup 3 > gpurun_out/r6/sp_lidar_front2.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/r6/sp_lidar_front2.log; exit 1; }
f=$(find /tmp/sp_lidar -name "*kernel_trace.csv" | head -1)
python tools/step_stats.py $f --marker pc2_count --steps 6 > gpurun_out/r6/step_stats_lidar_front2.txt || exit 1
head -40 gpurun_out/r6/step_stats_lidar_front2.txt
