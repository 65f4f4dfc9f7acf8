# Halo-tiled 3x3 pair kernels (tiles 90-93): GPU correctness tests, then the PointPillars backbone tile sweep.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_pair_storage_gpu.py -x -v -m gpu -k "halo" --timeout 120 --timeout-method thread > gpurun_out/hx_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/hx_tests.log | tail -20; tail -30 gpurun_out/hx_tests.log; exit 1; }
tail -1 gpurun_out/hx_tests.log
timeout -k 10 300 python tools/bench_conv_x3.py 0,71,95,96,97 pp.b1.conv --pair > gpurun_out/hx_tiles.jsonl 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/hx_tiles.jsonl; exit 1; }
cut -c1-420 gpurun_out/hx_tiles.jsonl
