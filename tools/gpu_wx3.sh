# wx3 (conv_hx3.hip Winograd F(2,3) along one axis): numerics tests, per-layer timing vs hx3.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_wx3.py -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/wx3_tests.log 2>&1 || { echo TESTS_FAILED; grep -E 'FAILED|Error|assert' gpurun_out/wx3_tests.log | head -20; tail -20 gpurun_out/wx3_tests.log; exit 1; }
tail -1 gpurun_out/wx3_tests.log
timeout -k 10 300 python -u tools/bench_conv_x3.py ${TILES:-110,130,131,132} ${LAYERS:-pp.b1.conv,pp.b2.conv,pp.b3.conv} --pair > gpurun_out/wx3_tiles.jsonl 2>&1 || { echo TILES_FAILED; tail -20 gpurun_out/wx3_tiles.jsonl; exit 1; }
cat gpurun_out/wx3_tiles.jsonl | grep layer
