# Per-layer F(2,3) A/B on one box: the current kernel build against the saved one
# (triton_client_amd/_lib/ab/libtca_kernels_base.so), fp32 / pair storage, 128- and 256-channel
# layers, alternating; the F(2,3) exactness tests of the current build first.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
TAG=${TAG:-micro}
mkdir -p gpurun_out/r6/$TAG
timeout -k 10 300 python -u -m pytest tests/test_wino_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/r6/$TAG/tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r6/$TAG/tests.log; exit 1; }
tail -1 gpurun_out/r6/$TAG/tests.log
BASE=$R/triton_client_amd/_lib/ab/libtca_kernels_base.so
for k in 1 2; do
  for L in new base; do
    if [ $L = base ]; then export TCA_KERNELS_LIB=$BASE; else unset TCA_KERNELS_LIB; fi
    for s in 1 2; do
      SHAPE=$s TILES=130 timeout -k 10 120 python tools/bench_wino.py > gpurun_out/r6/$TAG/b_${L}_s${s}_$k.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/r6/$TAG/b_${L}_s${s}_$k.log; exit 1; }
      echo "$L s$s run $k: $(tail -1 gpurun_out/r6/$TAG/b_${L}_s${s}_$k.log | cut -c30-200)"
    done
  done
done
unset TCA_KERNELS_LIB
