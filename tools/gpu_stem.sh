# fused K1 + stem + b1: tests, camera-only bench (fused vs chain)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_stem_fused_gpu.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/stem_tests.log 2>&1 || { echo TESTS_FAILED; grep -E 'FAILED|Error|assert' gpurun_out/stem_tests.log | head -20; tail -30 gpurun_out/stem_tests.log; exit 1; }
tail -1 gpurun_out/stem_tests.log
timeout -k 10 300 python bench.py --only camera --steps 30 --warmup 5 > gpurun_out/stem_bench_fused.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/stem_bench_fused.log; exit 1; }
tail -1 gpurun_out/stem_bench_fused.log | cut -c1-200
TCA_STEM_FUSED=0 timeout -k 10 300 python bench.py --only camera --steps 30 --warmup 5 > gpurun_out/stem_bench_chain.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/stem_bench_chain.log; exit 1; }
tail -1 gpurun_out/stem_bench_chain.log | cut -c1-200
