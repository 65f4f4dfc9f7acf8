# Pipelined step (--lidar-pipeline 3) vs the fused neck's persistent grid (TCA_NECK_GRID workgroups;
# 0 = one per CU) and the LiDAR-front stream priority, alternating.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
for k in 1 2; do
for v in "0 0" "128 0" "64 0" "0 1"; do
  set -- $v
  TCA_NECK_GRID=$1 timeout -k 10 300 python bench.py --steps 50 --warmup 10 --lidar-priority $2 > gpurun_out/ng_$1_$2.log 2>&1 || { echo BENCH_FAILED $v; tail -30 gpurun_out/ng_$1_$2.log; exit 1; }
  echo "grid=$1 prio=$2 $(tail -1 gpurun_out/ng_$1_$2.log | cut -c100-200)"
done
done
