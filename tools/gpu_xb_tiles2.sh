# 4-wave xb tiles (78, 79): bit identity, sweep on the PointPillars shapes, PMC of tile 70 vs 78 on pp.b2.conv.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 400 python -u -m pytest tests/test_pair_storage_gpu.py -x -v -m gpu -k "xb_bit" --timeout 200 --timeout-method thread > gpurun_out/xb2_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error" gpurun_out/xb2_tests.log | tail -20; tail -30 gpurun_out/xb2_tests.log; exit 1; }
tail -1 gpurun_out/xb2_tests.log
timeout -k 10 500 python tools/bench_conv_x3.py 70,78,71,79,73,77 pp --pair > gpurun_out/xb2_tiles.jsonl 2> gpurun_out/xb2_tiles.err || { echo FAILED; tail -20 gpurun_out/xb2_tiles.err; exit 1; }
cut -c1-500 gpurun_out/xb2_tiles.jsonl
LAYER=pp.b2.conv TILE=70 PREC=fp32p bash tools/gpu_conv_pmc.sh && LAYER=pp.b2.conv TILE=78 PREC=fp32p bash tools/gpu_conv_pmc.sh || exit 1
for t in 70 78; do python tools/pmc_summary.py conv_xb gpurun_out/pmc/pp.b2.conv_${t}_fp32p_p*.csv > gpurun_out/pmc_xb_$t.md; tail -5 gpurun_out/pmc_xb_$t.md; done
