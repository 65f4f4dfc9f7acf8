# Step-tail A/B: batched D2H-stage copy kernel (TCA_STAGE_COPY) and the 8-block NMS reduce
# (TCA_NMS_RB=8), after the rotated-NMS GPU tests under RB=8.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
TCA_NMS_RB=8 timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "nms" > gpurun_out/tail_nms_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/tail_nms_tests.log; exit 1; }
tail -1 gpurun_out/tail_nms_tests.log
for k in 1 2; do
for v in "0 4" "1 4" "1 8"; do
  set -- $v
  TCA_STAGE_COPY=$1 TCA_NMS_RB=$2 timeout -k 10 300 python bench.py --steps 50 --warmup 10 > gpurun_out/tail_$1_$2.log 2>&1 || { echo BENCH_FAILED $v; tail -30 gpurun_out/tail_$1_$2.log; exit 1; }
  echo "copy=$1 rb=$2 $(tail -1 gpurun_out/tail_$1_$2.log | cut -c100-200) 3d=$(grep -o '"avg_3d_dets_per_frame": [0-9.]*' gpurun_out/tail_$1_$2.log)"
done
done
cd /tmp && export TMPDIR=/tmp && cd $R
rm -rf /tmp/tail_full
TCA_NMS_RB=8 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/tail_full -o run -- python bench.py --steps 8 --warmup 3 > gpurun_out/tail_full.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/tail_full.log; exit 1; }
f=$(find /tmp/tail_full -name "*kernel_trace.csv" | head -1)
python tools/step_stats.py $f --marker yolo_stem --steps 6 --sequence > gpurun_out/tail_full_steps.txt || exit 1
head -40 gpurun_out/tail_full_steps.txt
