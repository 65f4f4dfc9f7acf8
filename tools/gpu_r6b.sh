# Round 6: voxeliser run-aggregated atomics + PointCloud2 aligned loads: the exactness tests, then a
# same-box A/B against the saved base build (tools/gpu_kernels_ab.sh) and LiDAR step kernel stats.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6
cd $R
TESTS="tests/test_ops_gpu.py tests/test_fp32_mode_gpu.py tests/test_pipelines_gpu.py" KSEL="voxel or pc2 or lidar or pillar or fp32" TAG=vox RUNS=2 bash tools/gpu_kernels_ab.sh || exit 1
cd /tmp && export TMPDIR=/tmp && cd $R
rm -rf /tmp/sp_lidar
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/sp_lidar -o run -- python bench.py --only lidar --steps 8 --warmup 3 > gpurun_out/r6/sp_lidar_vox.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/r6/sp_lidar_vox.log; exit 1; }
f=$(find /tmp/sp_lidar -name "*kernel_trace.csv" | head -1)
python tools/step_stats.py $f --marker pc2_count --steps 6 > gpurun_out/r6/step_stats_lidar_vox.txt || exit 1
head -40 gpurun_out/r6/step_stats_lidar_vox.txt
SHAPE=2 TILES=132,134 F32=1 timeout -k 10 200 python tools/bench_wino.py > gpurun_out/r6/bench_wino_256.log 2>&1 || { echo WINO_FAILED; tail -20 gpurun_out/r6/bench_wino_256.log; exit 1; }
cat gpurun_out/r6/bench_wino_256.log | tail -3
