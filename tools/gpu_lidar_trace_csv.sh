# LiDAR-only kernel trace CSV of a short bench run, copied back whole (per-dispatch grid sizes and times).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp && cd $R
mkdir -p gpurun_out/r6/voxtrace
rm -rf /tmp/vt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/vt -o run -- python bench.py --only lidar --steps 8 --warmup 3 > gpurun_out/r6/voxtrace/run.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/r6/voxtrace/run.log; exit 1; }
f=$(find /tmp/vt -name "*kernel_trace.csv" | head -1)
cp $f gpurun_out/r6/voxtrace/kernel_trace.csv
ls -la gpurun_out/r6/voxtrace/
