# Round 6: the persistent F(2,3) kernel (tca_conv_winop): exactness tests (bit-identical to the
# two-workgroup kernel, fp64 bound), then per-layer times against the default kernel on fp32 storage.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/r6/winop
timeout -k 10 300 python -u -m pytest tests/test_wino_gpu.py -x -v -m gpu -k "winop" --timeout 60 --timeout-method thread > gpurun_out/r6/winop/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r6/winop/tests.log; exit 1; }
tail -1 gpurun_out/r6/winop/tests.log
for s in 1 2 1 2; do
  F32=1 SHAPE=$s TILES=130,137,138 timeout -k 10 120 python tools/bench_wino.py >> gpurun_out/r6/winop/bench.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/r6/winop/bench.log; exit 1; }
  tail -1 gpurun_out/r6/winop/bench.log
done
