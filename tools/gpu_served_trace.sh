# Served path, round 5: kernel + copy trace of every process of the 4 + 4 client shm run.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5/srvtrace
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $R/gpurun_out/r5/srvtrace \
  -o %pid% -- python3 $R/tools/served_bench.py --frames 256 --window 8 --client-procs 4 --workers 96 --wire shm \
  --json-out $R/gpurun_out/r5/served_trace.json > $R/gpurun_out/r5/served_trace.log 2>&1 || { echo FAILED; tail -30 $R/gpurun_out/r5/served_trace.log; exit 1; }
tail -1 $R/gpurun_out/r5/served_trace.log | cut -c1-300
find $R/gpurun_out/r5/srvtrace -name "*.csv" | head -40
du -sh $R/gpurun_out/r5/srvtrace
