# LiDAR-only bench with / without double-buffered graph inputs, then the multi-rank gloo rehearsal.
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
for a in "" "--single-input-set" "" "--single-input-set"; do
  timeout -k 10 300 python bench.py --only lidar --steps 30 --warmup 5 $a > gpurun_out/lidab.log 2>&1 || { echo FAIL; tail -20 gpurun_out/lidab.log; exit 1; }
  echo "lidar [$a] $(tail -1 gpurun_out/lidab.log | cut -c100-200)"
done
bash tools/gpu_dp_rehearsal.sh
