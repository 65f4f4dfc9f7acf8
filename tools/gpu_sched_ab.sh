# Branch scheduling A/B on the headline (all with double-buffered graph inputs): fork graph (default)
# vs split graphs with / without the LiDAR stream at high priority; alternating, two rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
for k in 1 2; do
for cfg in "" "--graph-mode split --lidar-priority 1" "--graph-mode split"; do
  timeout -k 10 300 python bench.py --steps 50 --warmup 10 $cfg > gpurun_out/sched.log 2>&1 || { echo BENCH_FAILED "$cfg"; tail -20 gpurun_out/sched.log; exit 1; }
  echo "[$cfg] $(tail -1 gpurun_out/sched.log | cut -c100-200) $(grep -o '"graph_input_sets": [0-9]' gpurun_out/sched.log)"
done
done
