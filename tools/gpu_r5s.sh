# Round 5: F(2,3) on the 64-channel layers too (TCA_WINO_MIN_N=64) vs the default (128), three runs each.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5
cd $R
for k in 1 2 3; do
  for n in 128 64; do
    TCA_WINO_MIN_N=$n timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/r5/mn${n}_$k.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/r5/mn${n}_$k.log; exit 1; }
    echo "min_n=$n run $k: $(tail -1 gpurun_out/r5/mn${n}_$k.log | cut -c100-190)"
  done
done
