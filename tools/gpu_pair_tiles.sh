# Pair-storage split-product tiles on the PointPillars backbone shapes (batch 32).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 500 python tools/bench_conv_x3.py 20,25,26,32,50,51,52,53 pp --pair > gpurun_out/pair_tiles.jsonl 2> gpurun_out/pair_tiles.err || { echo FAILED; tail -20 gpurun_out/pair_tiles.err; exit 1; }
cat gpurun_out/pair_tiles.jsonl | cut -c1-600
