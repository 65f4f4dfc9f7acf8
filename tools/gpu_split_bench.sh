# Per-branch numbers for BASELINE.md: camera only / LiDAR only at batch 16 and batch 1 (streaming latency).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
for cfg in "camera 16" "lidar 16" "camera 1" "lidar 1"; do
  set -- $cfg
  timeout -k 10 240 python bench.py --steps 100 --warmup 10 --only $1 --batch $2 > gpurun_out/split_$1_$2.log 2>&1 || { echo FAILED $1 $2; tail -20 gpurun_out/split_$1_$2.log; exit 1; }
  echo "$1 $2: $(tail -1 gpurun_out/split_$1_$2.log | cut -c1-200)"
done
