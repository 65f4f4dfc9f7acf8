# Round 3 batch 1: hx3 probe + tests + per-layer tiles, then the new GPU tests
# (sweeps, served fp32 Detectron, DP families, rotated NMS replay).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 240 python tools/hx3_debug.py > gpurun_out/hx3_debug.log 2>&1 || { echo PROBE_FAILED; tail -20 gpurun_out/hx3_debug.log; }
tail -4 gpurun_out/hx3_debug.log
timeout -k 10 600 python -u -m pytest tests/test_hx3_gpu.py tests/test_centerpoint.py tests/test_ops_gpu.py tests/test_detectron.py "tests/test_fp32_mode_gpu.py::test_pipeline_fp32_detection_parity_headline_shape" -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/r3b1_tests.log 2>&1
echo "tests rc=$?"
grep -E "passed|failed" gpurun_out/r3b1_tests.log | tail -3
grep -E "^FAILED" gpurun_out/r3b1_tests.log | head -20
timeout -k 10 300 python -u tools/bench_conv_x3.py 90,94,96,97,110,111,112,113,114 pp.b1.conv,pp.b2.conv,pp.b3.conv --pair > gpurun_out/hx3_tiles.jsonl 2>&1 || { echo TILES_FAILED; tail -5 gpurun_out/hx3_tiles.jsonl; exit 1; }
grep layer gpurun_out/hx3_tiles.jsonl | cut -c1-250
