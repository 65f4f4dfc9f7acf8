set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $R && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/hp -o run -- python bench.py --steps 8 --warmup 3 $EXTRA > gpurun_out/hp.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/hp.log; exit 1; }
f=$(find /tmp/hp -name "*kernel_trace.csv" | head -1)
python tools/trace_tail.py $f 400 > gpurun_out/headline_tail.txt
