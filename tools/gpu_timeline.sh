# Full headline step (default flags) kernel trace with per-dispatch start / end offsets and queues.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $R
rm -rf /tmp/tl_full
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/tl_full -o run -- python bench.py --steps 8 --warmup 3 $EXTRA > gpurun_out/tl_full.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/tl_full.log; exit 1; }
f=$(find /tmp/tl_full -name "*kernel_trace.csv" | head -1)
python tools/step_stats.py $f --marker ${MARKER:-pc2_count} --steps 6 --sequence > gpurun_out/tl_full_steps.txt || exit 1
head -3 gpurun_out/tl_full_steps.txt
