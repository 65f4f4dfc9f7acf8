# Round 5: neck A/B (standalone, variants 0 and 1), neck PMC, LiDAR per-layer table; then the remote parts.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5
cd $R
timeout -k 10 300 python tools/bench_neck.py 32 0,1 > gpurun_out/r5/neck_ab.log 2>&1 || { echo NECK_AB_FAILED; tail -20 gpurun_out/r5/neck_ab.log; exit 1; }
tail -1 gpurun_out/r5/neck_ab.log
timeout -k 10 300 python tools/layer_times.py --branch lidar --batch 32 > gpurun_out/r5/layers_lidar.txt 2>&1 || { echo LAYERS_FAILED; tail -20 gpurun_out/r5/layers_lidar.txt; exit 1; }
head -30 gpurun_out/r5/layers_lidar.txt
bash tools/gpu_neck_pmc.sh > gpurun_out/r5/neck_pmc.txt 2>&1 || { echo PMC_FAILED; tail -20 gpurun_out/r5/neck_pmc.txt; exit 1; }
cat gpurun_out/pmc_neck_r5.md | tail -8
bash tools/gpu_r5a.sh > gpurun_out/r5/part_a.txt 2>&1 || { echo A_PART_FAILED; tail -30 gpurun_out/r5/part_a.txt; exit 1; }
cat gpurun_out/r5/part_a.txt | cut -c1-300
bash tools/gpu_r5b.sh > gpurun_out/r5/part_b.txt 2>&1 || { echo B_PART_FAILED; tail -30 gpurun_out/r5/part_b.txt; exit 1; }
cat gpurun_out/r5/part_b.txt | cut -c1-400 | head -40
