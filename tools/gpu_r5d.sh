# Round 5: neck v1 PMC, LiDAR-step PMC (every kernel), then the remote parts and the step profile.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5
cd $R
sed -i 's/bench_neck.py 32 0/bench_neck.py 32 1/' tools/gpu_neck_pmc.sh
bash tools/gpu_neck_pmc.sh > gpurun_out/r5/neck_pmc.txt 2>&1 || { echo PMC_FAILED; tail -20 gpurun_out/r5/neck_pmc.txt; exit 1; }
tail -7 gpurun_out/pmc_neck_r5.md
bash tools/gpu_lidar_pmc.sh > gpurun_out/r5/lidar_pmc.txt 2>&1 || { echo LPMC_FAILED; tail -20 gpurun_out/r5/lidar_pmc.txt; exit 1; }
for k in conv_hx3_kernel conv_hx3s2_kernel pillar_vfe anchor_decode nms_mask_rot vox_fill; do echo "== $k"; python tools/pmc_summary.py $k gpurun_out/pmc_lidar/p*.csv | tail -6; done
bash tools/gpu_r5a.sh > gpurun_out/r5/part_a.txt 2>&1 || { echo A_PART_FAILED; tail -30 gpurun_out/r5/part_a.txt; exit 1; }
cat gpurun_out/r5/part_a.txt | cut -c1-300
bash tools/gpu_r5b.sh > gpurun_out/r5/part_b.txt 2>&1 || { echo B_PART_FAILED; tail -30 gpurun_out/r5/part_b.txt; exit 1; }
cat gpurun_out/r5/part_b.txt | cut -c1-400 | head -40
