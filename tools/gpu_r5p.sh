# Round 5: conv_wino direct-store epilogue A/B (TCA_WINO_DBG=8) + numerics with it.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5
cd $R
TCA_WINO_DBG=8 timeout -k 10 300 python -u -m pytest tests/test_wino_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/r5/wino_tests8.log 2>&1 || { echo WINO_TESTS_FAILED; tail -30 gpurun_out/r5/wino_tests8.log; exit 1; }
tail -1 gpurun_out/r5/wino_tests8.log
for k in 1 2; do
for d in 0 8; do
  for sh in 1 2; do
    TCA_WINO_DBG=$d F32=1 SHAPE=$sh TILES=132 timeout -k 10 120 python tools/bench_wino.py > gpurun_out/r5/wdbg_$d.log 2>&1 || { echo FAILED $d; tail -5 gpurun_out/r5/wdbg_$d.log; exit 1; }
    echo "dbg=$d $(tail -1 gpurun_out/r5/wdbg_$d.log)"
  done
done
done
