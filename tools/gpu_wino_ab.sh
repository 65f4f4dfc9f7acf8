# Round 5: headline A/B on one box: F(2,3) on every stride-1 layer / N >= 128 only / off.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5
cd $R
timeout -k 10 200 python tools/bench_wino.py > gpurun_out/r5/bench_wino_n.log 2>&1 || { echo BENCH_WINO_FAILED; tail -20 gpurun_out/r5/bench_wino_n.log; exit 1; }
cat gpurun_out/r5/bench_wino_n.log | cut -c1-250
for k in 1 2; do
  for cfg in "1 64" "1 128" "0 64"; do
    set -- $cfg
    TCA_WINO=$1 TCA_WINO_MIN_N=$2 timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/r5/abn_w$1_n$2_$k.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/r5/abn_w$1_n$2_$k.log; exit 1; }
    echo "wino=$1 min_n=$2 run $k: $(tail -1 gpurun_out/r5/abn_w$1_n$2_$k.log | cut -c100-190)"
  done
done
