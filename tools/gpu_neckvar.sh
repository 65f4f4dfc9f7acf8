# Pipelined step vs the fused neck's footprint: variant (TCA_NECK_VARIANT: 0 auto <8 waves>, 2 <4 waves>,
# launched 2 x grid) and persistent grid (TCA_NECK_GRID), alternating x2.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
for k in 1 2; do
for v in "0 0" "2 128" "2 64"; do
  set -- $v
  TCA_NECK_VARIANT=$1 TCA_NECK_GRID=$2 timeout -k 10 300 python bench.py --steps 50 --warmup 10 > gpurun_out/nv_$1_$2.log 2>&1 || { echo BENCH_FAILED $v; tail -30 gpurun_out/nv_$1_$2.log; exit 1; }
  echo "variant=$1 grid=$2 $(tail -1 gpurun_out/nv_$1_$2.log | cut -c100-200) 3d=$(grep -o '"avg_3d_dets_per_frame": [0-9.]*' gpurun_out/nv_$1_$2.log)"
done
done
