# Camera-only fp32 step, kernel trace in launch order (per-layer times of the YOLOv5n plan at batch 32).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $R
rm -rf /tmp/camseq
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/camseq -o run -- python bench.py --only camera --steps 8 --warmup 3 > gpurun_out/camseq.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/camseq.log; exit 1; }
f=$(find /tmp/camseq -name "*kernel_trace.csv" | head -1)
head -1 $f > gpurun_out/camseq_header.txt
python tools/step_stats.py $f --marker ${MARKER:-yolo_stem} --steps 6 --sequence > gpurun_out/camseq_steps.txt || exit 1
head -3 gpurun_out/camseq_steps.txt
