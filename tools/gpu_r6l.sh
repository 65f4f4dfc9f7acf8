# Round 6, served path: (1) the 4 + 4 client shm run under a kernel + memory-copy + HIP API trace,
# every copyBuffer blit joined to the API call that issued it (tools/copybuffer_origin.py);
# (2) untraced served runs over devshm and shm with the server stage clock (tools/gpu_served3.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/r6/served
cd /tmp && export TMPDIR=/tmp && cd $R
rm -rf /tmp/srvtrace
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d /tmp/srvtrace \
  -o %pid% -- python3 tools/served_bench.py --frames 128 --window 8 --client-procs 4 --workers 32 --wire shm \
  --json-out gpurun_out/r6/served/served_trace.json > gpurun_out/r6/served/served_trace.log 2>&1 || { echo TRACE_FAILED; grep -v "^W2026" gpurun_out/r6/served/served_trace.log | tail -30; exit 1; }
tail -1 gpurun_out/r6/served/served_trace.log | cut -c1-300
D=$(dirname $(find /tmp/srvtrace -name "*_kernel_trace.csv" | head -1))
python tools/copybuffer_origin.py $D > gpurun_out/r6/served/copybuffer_origin.txt || exit 1
head -30 gpurun_out/r6/served/copybuffer_origin.txt
python tools/served_trace_summary.py $D > gpurun_out/r6/served/trace_summary.txt || exit 1
cat gpurun_out/r6/served/trace_summary.txt
NOTEST=1 WIRES="devshm shm" TAG=_r6 bash tools/gpu_served3.sh
