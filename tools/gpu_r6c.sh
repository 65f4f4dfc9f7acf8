# Round 6: upper bounds for the LiDAR front (tools/whatif_bench.py, diagnostic only): the headline
# with the voxeliser / the whole front removed from the captured step, beside the default, one box.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6/whatif
cd $R
for k in 1 2; do
  for m in default novox nofront; do
    W=$m; [ $m = default ] && W=
    WHATIF=$W timeout -k 10 300 python tools/whatif_bench.py --steps 30 --warmup 5 > gpurun_out/r6/whatif/$m.$k.log 2>&1 || { echo WHATIF_FAILED $m; tail -20 gpurun_out/r6/whatif/$m.$k.log; exit 1; }
    echo "$m $k: $(tail -1 gpurun_out/r6/whatif/$m.$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  done
done
