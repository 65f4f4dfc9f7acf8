# Double-buffered graph inputs vs one input set + D2D copy: headline A/B, gloo 2-rank rehearsal, camera-only.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
for k in 1 2; do
  timeout -k 10 300 python bench.py --steps 50 --warmup 10 > gpurun_out/dbuf_on_$k.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/dbuf_on_$k.log; exit 1; }
  echo "2 sets $(tail -1 gpurun_out/dbuf_on_$k.log | cut -c100-200)"
  timeout -k 10 300 python bench.py --steps 50 --warmup 10 --single-input-set > gpurun_out/dbuf_off_$k.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/dbuf_off_$k.log; exit 1; }
  echo "1 set  $(tail -1 gpurun_out/dbuf_off_$k.log | cut -c100-200)"
done
grep -o '"graph_input_sets": [0-9]' gpurun_out/dbuf_on_1.log
timeout -k 10 300 python bench.py --only lidar --steps 10 --warmup 3 > gpurun_out/dbuf_lidar.log 2>&1 || { echo BENCH_FAILED lidar; tail -20 gpurun_out/dbuf_lidar.log; exit 1; }
echo "lidar only $(tail -1 gpurun_out/dbuf_lidar.log | cut -c100-200)"
