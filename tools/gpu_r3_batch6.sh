# Round 3 batch 6: stride-2 hx3 (phase kernel): tests, per-layer timing vs the xb tiles, step profile.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_hx3_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r3b6_tests.log 2>&1 || { echo TESTS_FAILED; grep -E 'FAILED|Error|assert' gpurun_out/r3b6_tests.log | head -20; tail -20 gpurun_out/r3b6_tests.log; exit 1; }
tail -1 gpurun_out/r3b6_tests.log
timeout -k 10 300 python -u tools/bench_conv_x3.py 73,77,120,121,122,123,124 pp.b1.down,pp.b2.down,pp.b3.down --pair > gpurun_out/hx3s2_tiles.jsonl 2>&1 || { echo TILES_FAILED; tail -20 gpurun_out/hx3s2_tiles.jsonl; exit 1; }
grep layer gpurun_out/hx3s2_tiles.jsonl | cut -c1-220
TAG=r3_s2 bash tools/gpu_step_profile.sh
