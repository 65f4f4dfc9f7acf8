set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_hx3_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r3b3_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error" gpurun_out/r3b3_tests.log | head; exit 1; }
tail -1 gpurun_out/r3b3_tests.log
timeout -k 10 300 python -u tools/bench_conv_x3.py 96,110,111,112,113,114,115,116 pp.b1.conv,pp.b2.conv,pp.b3.conv --pair > gpurun_out/hx3_tiles2.jsonl 2>&1 || { echo TILES_FAILED; tail -5 gpurun_out/hx3_tiles2.jsonl; exit 1; }
grep layer gpurun_out/hx3_tiles2.jsonl | cut -c1-220
