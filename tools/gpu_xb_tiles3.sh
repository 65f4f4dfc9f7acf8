# One-wave-column pair xb tiles (68, 69) on the N=64 PointPillars layers vs 71 / 77, with bit identity.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_pair_storage_gpu.py -x -v -m gpu -k "xb_bit" --timeout 200 --timeout-method thread > gpurun_out/xb3_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error" gpurun_out/xb3_tests.log | tail -20; tail -30 gpurun_out/xb3_tests.log; exit 1; }
tail -1 gpurun_out/xb3_tests.log
timeout -k 10 500 python tools/bench_conv_x3.py 71,68,77,69 pp.b1 --pair > gpurun_out/xb3_tiles.jsonl 2> gpurun_out/xb3_tiles.err || { echo FAILED; tail -20 gpurun_out/xb3_tiles.err; exit 1; }
cut -c1-400 gpurun_out/xb3_tiles.jsonl
