# Round 5: conv_wino position-wise U registers: tests, per-layer A/B, headline A/B (all layers /
# N >= 128 only / off).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5
cd $R
timeout -k 10 300 python -u -m pytest tests/test_wino_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5/wino_tests.log 2>&1 || { echo WINO_TESTS_FAILED; tail -30 gpurun_out/r5/wino_tests.log; exit 1; }
tail -1 gpurun_out/r5/wino_tests.log
timeout -k 10 600 python -u -m pytest tests/test_bev_uniform_gpu.py tests/test_fp32_mode_gpu.py tests/test_hx3_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r5/wino_fp32_tests.log 2>&1 || { echo FP32_TESTS_FAILED; tail -30 gpurun_out/r5/wino_fp32_tests.log; exit 1; }
tail -1 gpurun_out/r5/wino_fp32_tests.log
timeout -k 10 200 python tools/bench_wino.py > gpurun_out/r5/bench_wino.log 2>&1 || { echo BENCH_WINO_FAILED; tail -20 gpurun_out/r5/bench_wino.log; exit 1; }
cat gpurun_out/r5/bench_wino.log
for k in 1 2; do
  for cfg in "1 64" "1 128" "0 64"; do
    set -- $cfg
    TCA_WINO=$1 TCA_WINO_MIN_N=$2 timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/r5/ab_w$1_n$2_$k.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/r5/ab_w$1_n$2_$k.log; exit 1; }
    echo "wino=$1 min_n=$2 run $k: $(tail -1 gpurun_out/r5/ab_w$1_n$2_$k.log | cut -c100-190)"
  done
done
