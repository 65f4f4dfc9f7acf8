# Per-layer F(2,3) times (bench_wino.py) for the current kernel build and the saved one
# (triton_client_amd/_lib/ab/libtca_kernels_base.so), alternating, then the headline A/B
# (gpu_kernels_ab.sh).  TAG names the logs.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-wlab}
mkdir -p $R/gpurun_out/r5
cd $R
for k in 1 2; do
  for L in new base; do
    if [ $L = base ]; then export TCA_KERNELS_LIB=$R/triton_client_amd/_lib/ab/libtca_kernels_base.so; else unset TCA_KERNELS_LIB; fi
    TCA_WINO_MIN_N=64 TILES=130,132 timeout -k 10 200 python tools/bench_wino.py > gpurun_out/r5/${TAG}_w_${L}_$k.log 2>&1 || { echo WINO_FAILED; tail -20 gpurun_out/r5/${TAG}_w_${L}_$k.log; exit 1; }
    echo "$L $k: $(python3 -c "import json,sys; [print(d[\"shape\"][3], {k: v[\"us\"] for k, v in d.items() if isinstance(v, dict)}) for d in map(json.loads, (l for l in open(sys.argv[1]) if l.startswith(\"{\")))]" gpurun_out/r5/${TAG}_w_${L}_$k.log | tr "\n" " ")"
  done
done
unset TCA_KERNELS_LIB
TAG=$TAG RUNS=${RUNS:-2} bash tools/gpu_kernels_ab.sh
