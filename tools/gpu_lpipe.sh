# LiDAR software pipeline A/B (--lidar-pipeline 1 vs 0): headline x2 alternating, LiDAR only, and a 2-rank
# gloo rehearsal of the pipelined path.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
for k in 1 2; do
for p in 1 0; do
  timeout -k 10 300 python bench.py --steps 50 --warmup 10 --lidar-pipeline $p > gpurun_out/lpipe_$p.log 2>&1 || { echo BENCH_FAILED $p; tail -30 gpurun_out/lpipe_$p.log; exit 1; }
  echo "pipeline=$p $(tail -1 gpurun_out/lpipe_$p.log | cut -c100-200) $(grep -o '"lidar_pipelined": [a-z]*' gpurun_out/lpipe_$p.log) 3d=$(grep -o '"avg_3d_dets_per_frame": [0-9.]*' gpurun_out/lpipe_$p.log)"
done
done
timeout -k 10 300 python bench.py --only lidar --steps 30 --warmup 5 --lidar-pipeline 1 > gpurun_out/lpipe_lid.log 2>&1 || { echo BENCH_FAILED lid; tail -30 gpurun_out/lpipe_lid.log; exit 1; }
echo "lidar only pipelined $(tail -1 gpurun_out/lpipe_lid.log | cut -c100-200)"
export TCA_DIST_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --steps 5 --warmup 2 --lidar-pipeline 1 > gpurun_out/lpipe_dp2.log 2>&1 || { echo DP_FAILED; tail -30 gpurun_out/lpipe_dp2.log; exit 1; }
echo "dp2 $(grep '^{' gpurun_out/lpipe_dp2.log | cut -c100-200) 3d=$(grep -o '"avg_3d_dets_per_frame": [0-9.]*' gpurun_out/lpipe_dp2.log)"
