# hx3 (conv_hx3.hip): numerics tests, per-layer timing vs the conv_mfma.hip halo tiles, LiDAR bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_hx3_gpu.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/hx3_tests.log 2>&1 || { echo TESTS_FAILED; grep -E 'FAILED|Error|assert' gpurun_out/hx3_tests.log | head -20; tail -20 gpurun_out/hx3_tests.log; exit 1; }
tail -1 gpurun_out/hx3_tests.log
timeout -k 10 300 python -u tools/bench_conv_x3.py 90,94,96,97,110,111,112,113,114 pp.b1.conv,pp.b2.conv,pp.b3.conv --pair > gpurun_out/hx3_tiles.jsonl 2>&1 || { echo TILES_FAILED; tail -20 gpurun_out/hx3_tiles.jsonl; exit 1; }
cat gpurun_out/hx3_tiles.jsonl | grep layer
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/hx3_bench.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/hx3_bench.log; exit 1; }
tail -1 gpurun_out/hx3_bench.log | cut -c1-300
