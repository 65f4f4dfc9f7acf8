# Round 5: same-box A/B of the headline with F(2,3) stride-1 convs on / off (TCA_WINO), twice each.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5
cd $R
for k in 1 2; do
  for w in 1 0; do
    TCA_WINO=$w timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/r5/ab_wino${w}_$k.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/r5/ab_wino${w}_$k.log; exit 1; }
    echo "wino=$w run $k: $(tail -1 gpurun_out/r5/ab_wino${w}_$k.log | cut -c1-200)"
  done
done
