# Same-box kernel tables of the headline step with and without the voxeliser chain (WHATIF=novox, diagnostic):
# which kernels the chain slows down when it runs beside them.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/r6/whatif_trace
cd /tmp && export TMPDIR=/tmp && cd $R
for m in none novox; do
  if [ $m = none ]; then unset WHATIF; else export WHATIF=$m; fi
  rm -rf /tmp/wt_$m
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/wt_$m -o run -- python tools/whatif_bench.py --steps 8 --warmup 3 > gpurun_out/r6/whatif_trace/$m.log 2>&1 || { echo PROF_FAILED $m; tail -20 gpurun_out/r6/whatif_trace/$m.log; exit 1; }
  f=$(find /tmp/wt_$m -name "*kernel_trace.csv" | head -1)
  python tools/step_stats.py $f --marker ${MARKER:-yolo_stem} --steps 6 > gpurun_out/r6/whatif_trace/stats_$m.txt || exit 1
  echo "== $m"; head -40 gpurun_out/r6/whatif_trace/stats_$m.txt
done
unset WHATIF
