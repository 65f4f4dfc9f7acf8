# hx3 PAIRS (two static weight sets, no register copies) vs the copy loop: tests, per-layer timing.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_hx3_gpu.py -x -q -m gpu --timeout 200 --timeout-method thread > gpurun_out/r3b5_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error" gpurun_out/r3b5_tests.log | head; exit 1; }
tail -1 gpurun_out/r3b5_tests.log
for p in 1 0; do
  TCA_HX3_PAIRS=$p timeout -k 10 300 python -u tools/bench_conv_x3.py 110 pp.b1.conv,pp.b2.conv,pp.b3.conv --pair > gpurun_out/hx3_pairs$p.jsonl 2>&1 || { echo TILES_FAILED; tail -5 gpurun_out/hx3_pairs$p.jsonl; exit 1; }
  echo "PAIRS=$p"; grep layer gpurun_out/hx3_pairs$p.jsonl | cut -c1-160
done
