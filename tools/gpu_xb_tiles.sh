# Buffer-descriptor pair conv (xb, tiles 70-77): bit identity vs the glds twins, then the tile sweep
# on the PointPillars backbone shapes (batch 32) next to the glds tiles.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_pair_storage_gpu.py -x -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/xb_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error" gpurun_out/xb_tests.log | tail -20; tail -30 gpurun_out/xb_tests.log; exit 1; }
tail -1 gpurun_out/xb_tests.log
timeout -k 10 500 python tools/bench_conv_x3.py 25,70,74,26,71,75,32,72,20,73,37,76,22,77 pp --pair > gpurun_out/xb_tiles.jsonl 2> gpurun_out/xb_tiles.err || { echo FAILED; tail -20 gpurun_out/xb_tiles.err; exit 1; }
cut -c1-700 gpurun_out/xb_tiles.jsonl
