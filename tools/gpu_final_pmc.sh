# The final tree's LiDAR-step PMC summary (tools/gpu_lidar_pmc.sh passes + tools/pmc_summary.py per
# kernel) -> gpurun_out/pmc_lidar/summary.md
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_lidar_pmc.sh || exit 1
: > gpurun_out/pmc_lidar/summary.md
for k in conv_wino bev_neck conv_hx3_kernel conv_hx3s2 pillar_vfe_lin nms_mask_rot; do
  echo "## $k" >> gpurun_out/pmc_lidar/summary.md
  python tools/pmc_summary.py $k gpurun_out/pmc_lidar/p*.csv | sed -n '/Derived/,$p' >> gpurun_out/pmc_lidar/summary.md || true
done
cat gpurun_out/pmc_lidar/summary.md
