# A/B of the current tree against an older commit built in .ab_old (a git worktree), on one box.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r4
for rep in 1 2; do
  for v in old new; do
    D=$R; [ $v = old ] && D=$R/.ab_old
    for only in lidar both; do
      (cd $D && timeout -k 10 300 python bench.py --only $only --steps 30 --warmup 10) > $R/gpurun_out/r4/abo_${only}_${v}_$rep.log 2>&1 || { echo BENCH_FAILED $v; tail -20 $R/gpurun_out/r4/abo_${only}_${v}_$rep.log; exit 1; }
      echo "$rep $v $only $(tail -1 $R/gpurun_out/r4/abo_${only}_${v}_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
    done
  done
done
