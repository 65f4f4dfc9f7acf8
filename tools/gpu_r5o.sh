# Round 5: conv_wino bottleneck experiments (TCA_WINO_DBG switches), 128-channel layer, fp32 io.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5
cd $R
for d in 0 1 2 4 3 7; do
  TCA_WINO_DBG=$d F32=1 SHAPE=1 TILES=132 timeout -k 10 120 python tools/bench_wino.py > gpurun_out/r5/wdbg_$d.log 2>&1 || { echo FAILED $d; tail -5 gpurun_out/r5/wdbg_$d.log; exit 1; }
  echo "dbg=$d $(tail -1 gpurun_out/r5/wdbg_$d.log)"
done
for d in 0 1 2 4 3 7; do
  TCA_WINO_DBG=$d F32=1 SHAPE=2 TILES=132 timeout -k 10 120 python tools/bench_wino.py > gpurun_out/r5/wdbg2_$d.log 2>&1 || { echo FAILED $d; tail -5 gpurun_out/r5/wdbg2_$d.log; exit 1; }
  echo "256ch dbg=$d $(tail -1 gpurun_out/r5/wdbg2_$d.log)"
done
