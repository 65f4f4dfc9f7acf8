# Same-box headline A/B of an environment switch: VAR=name, A / B = its two values (default
# unset / 1), RUNS rounds alternating A and B; EXTRA = bench.py flags.  Logs: gpurun_out/r5/${TAG}_*.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-envab}
RUNS=${RUNS:-3}
mkdir -p $R/gpurun_out/r5
cd $R
val() { python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"; }
for k in $(seq 1 $RUNS); do
  for L in A B; do
    v=$A; [ $L = B ] && v=$B
    if [ -z "$v" ]; then unset $VAR; else export $VAR=$v; fi
    timeout -k 10 300 python bench.py --steps 30 --warmup 5 $EXTRA > gpurun_out/r5/${TAG}_${L}_$k.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/r5/${TAG}_${L}_$k.log; exit 1; }
    echo "$VAR=$v run $k: $(tail -1 gpurun_out/r5/${TAG}_${L}_$k.log | val)"
  done
done
