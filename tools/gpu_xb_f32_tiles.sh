# fp32-input xb twins (tiles 80-87): bit identity vs the glds tiles, then the camera-layer tile sweep (batch 32).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_pair_storage_gpu.py -x -v -m gpu -k "fp32_xb" --timeout 200 --timeout-method thread > gpurun_out/xbf_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error" gpurun_out/xbf_tests.log | tail -20; tail -30 gpurun_out/xbf_tests.log; exit 1; }
tail -1 gpurun_out/xbf_tests.log
timeout -k 10 500 python tools/bench_conv_x3.py 0,20,80,41,81,22,84,24,85,25,82,26,83,42,86 y > gpurun_out/xbf_tiles.jsonl 2> gpurun_out/xbf_tiles.err || { echo FAILED; tail -20 gpurun_out/xbf_tiles.err; exit 1; }
cut -c1-800 gpurun_out/xbf_tiles.jsonl
