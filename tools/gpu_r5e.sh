# Round 5: s2 halo double-buffering + pixel-major anchor decode: numerics, per-layer + step profile; remote parts.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5
cd $R
timeout -k 10 600 python -u -m pytest tests/test_hx3_gpu.py tests/test_ops_gpu.py tests/test_fp32_mode_gpu.py tests/test_pipelines_gpu.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/r5/e_tests.log 2>&1 || { echo TESTS_FAILED; grep -E 'FAILED|Error' gpurun_out/r5/e_tests.log | tail -30; tail -40 gpurun_out/r5/e_tests.log; exit 1; }
tail -1 gpurun_out/r5/e_tests.log
timeout -k 10 300 python tools/layer_times.py --branch lidar --batch 32 > gpurun_out/r5/layers_lidar_e.txt 2>&1 || { echo LAYERS_FAILED; tail -20 gpurun_out/r5/layers_lidar_e.txt; exit 1; }
head -6 gpurun_out/r5/layers_lidar_e.txt
TAG=r5e bash tools/gpu_step_profile.sh || exit 1
bash tools/gpu_r5a.sh > gpurun_out/r5/part_a.txt 2>&1 || { echo A_PART_FAILED; tail -30 gpurun_out/r5/part_a.txt; exit 1; }
cat gpurun_out/r5/part_a.txt | cut -c1-300
bash tools/gpu_r5b.sh > gpurun_out/r5/part_b.txt 2>&1 || { echo B_PART_FAILED; tail -30 gpurun_out/r5/part_b.txt; exit 1; }
cat gpurun_out/r5/part_b.txt | cut -c1-400 | head -40
