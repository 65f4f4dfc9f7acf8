# Per-dispatch launch-order tables of one camera and one LiDAR step (kernel trace).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $R
for br in camera lidar; do
  rm -rf /tmp/sq_$br
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/sq_$br -o run -- python bench.py --only $br --steps 6 --warmup 3 > gpurun_out/sq_$br.log 2>&1 || { echo PROF_FAILED $br; tail -20 gpurun_out/sq_$br.log; exit 1; }
  f=$(find /tmp/sq_$br -name "*kernel_trace.csv" | head -1)
  m=pc2_count; [ $br = camera ] && m=prep_
  python tools/step_stats.py $f --marker $m --steps 4 --sequence > gpurun_out/seq_${br}_r3.txt || exit 1
  head -2 gpurun_out/seq_${br}_r3.txt
done
