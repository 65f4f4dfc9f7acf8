# Headline bench plus per-branch, setup-excluded kernel traces.
#   EXTRA: extra bench.py flags (e.g. "--precision bf16"); TAG: output suffix.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
TAG=${TAG:-r2}
cd $R
timeout -k 10 300 python bench.py --steps 50 --warmup 10 $EXTRA > gpurun_out/bench_$TAG.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/bench_$TAG.log; exit 1; }
tail -1 gpurun_out/bench_$TAG.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp && cd $R
for br in camera lidar; do
  rm -rf /tmp/sp_$br
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/sp_$br -o run -- python bench.py --only $br --steps 8 --warmup 3 $EXTRA > gpurun_out/sp_${br}_$TAG.log 2>&1 || { echo PROF_FAILED $br; tail -20 gpurun_out/sp_${br}_$TAG.log; exit 1; }
  f=$(find /tmp/sp_$br -name "*kernel_trace.csv" | head -1)
  m=pc2_count; [ $br = camera ] && m=${CAM_MARKER:-yolo_stem}
  python tools/step_stats.py $f --marker $m --steps 6 > gpurun_out/step_stats_${br}_$TAG.txt || exit 1
  head -3 gpurun_out/step_stats_${br}_$TAG.txt
done
