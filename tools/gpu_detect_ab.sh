# A/B of the fused Detect + filter kernel on one box: camera-only and headline, twice each.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r4
cd $R
for rep in 1 2; do
  for mode in unfused fused; do
    F=""; [ $mode = unfused ] && F="--unfused-detect"
    for only in camera both; do
      timeout -k 10 300 python bench.py --only $only --steps 30 --warmup 10 $F > gpurun_out/r4/dab_${only}_${mode}_$rep.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/r4/dab_${only}_${mode}_$rep.log; exit 1; }
      echo "$rep $mode $only $(tail -1 gpurun_out/r4/dab_${only}_${mode}_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
    done
  done
done
