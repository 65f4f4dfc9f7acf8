# A/B of the BEV 3x3 layers: the current tree against the commit built in .ab_old, on one box.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r4
for rep in 1 2; do
  for v in old new; do
    D=$R; [ $v = old ] && D=$R/.ab_old
    (cd $D && timeout -k 10 300 python tools/bench_conv_x3.py 0 pp.b1.conv,pp.b2.conv,pp.b3.conv --pair) > $R/gpurun_out/r4/abc_${v}_$rep.jsonl 2>&1 || { echo CONV_FAILED $v; tail -20 $R/gpurun_out/r4/abc_${v}_$rep.jsonl; exit 1; }
    echo "$rep $v $(grep -h '^{' $R/gpurun_out/r4/abc_${v}_$rep.jsonl | python -c 'import json,sys; print([(json.loads(l)["layer"], json.loads(l)["best_us"]) for l in sys.stdin])')"
  done
done
for v in old new; do
  D=$R; [ $v = old ] && D=$R/.ab_old
  (cd $D && timeout -k 10 300 python bench.py --only lidar --steps 30 --warmup 10) > $R/gpurun_out/r4/abc_lidar_$v.log 2>&1 || { echo BENCH_FAILED; exit 1; }
  echo "lidar $v $(tail -1 $R/gpurun_out/r4/abc_lidar_$v.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
