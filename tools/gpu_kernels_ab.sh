# Same-box A/B of the current kernel build against a saved one (TCA_KERNELS_LIB =
# triton_client_amd/_lib/ab/libtca_kernels_base.so): the GPU tests named by TESTS / KSEL first,
# then LiDAR-only and headline bench runs, RUNS rounds alternating new / base.  TAG names the logs.
set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-ab}
RUNS=${RUNS:-2}
mkdir -p $R/gpurun_out/r5 $R/gpurun_out/r6
cd $R
if [ -n "$TESTS" ]; then
  timeout -k 10 400 python -u -m pytest $TESTS -x -q -m gpu ${KSEL:+-k "$KSEL"} --timeout 200 --timeout-method thread > gpurun_out/r5/${TAG}_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r5/${TAG}_tests.log; exit 1; }
  tail -1 gpurun_out/r5/${TAG}_tests.log
fi
BASE=$R/triton_client_amd/_lib/ab/libtca_kernels_base.so
for k in $(seq 1 $RUNS); do
  for L in new base; do
    if [ $L = base ]; then export TCA_KERNELS_LIB=$BASE; [ -n "$BASE_ENV" ] && export $BASE_ENV; else unset TCA_KERNELS_LIB; [ -n "$BASE_ENV" ] && unset ${BASE_ENV%%=*}; fi
    timeout -k 10 300 python bench.py --only lidar --steps 30 --warmup 5 > gpurun_out/r5/${TAG}_l_${L}_$k.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/r5/${TAG}_l_${L}_$k.log; exit 1; }
    timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/r5/${TAG}_h_${L}_$k.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/r5/${TAG}_h_${L}_$k.log; exit 1; }
    echo "$L run $k: lidar $(tail -1 gpurun_out/r5/${TAG}_l_${L}_$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d[\"value\"], d[\"ms_per_step\"])") headline $(tail -1 gpurun_out/r5/${TAG}_h_${L}_$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d[\"value\"], d[\"ms_per_step\"])")"
  done
done
if [ -n "$STATS" ]; then  # same-box LiDAR step kernel tables of both builds
  cd /tmp && export TMPDIR=/tmp && cd $R
  for L in new base; do
    if [ $L = base ]; then export TCA_KERNELS_LIB=$BASE; [ -n "$BASE_ENV" ] && export $BASE_ENV; else unset TCA_KERNELS_LIB; [ -n "$BASE_ENV" ] && unset ${BASE_ENV%%=*}; fi
    rm -rf /tmp/ab_sp
    timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/ab_sp -o run -- python bench.py --only lidar --steps 8 --warmup 3 > gpurun_out/r6/${TAG}_sp_$L.log 2>&1 || { echo PROF_FAILED $L; tail -20 gpurun_out/r6/${TAG}_sp_$L.log; exit 1; }
    f=$(find /tmp/ab_sp -name "*kernel_trace.csv" | head -1)
    python tools/step_stats.py $f --marker pc2_count --steps 6 > gpurun_out/r6/${TAG}_stats_$L.txt || exit 1
    echo "== $L"; head -24 gpurun_out/r6/${TAG}_stats_$L.txt
  done
  unset TCA_KERNELS_LIB
  [ -n "$BASE_ENV" ] && unset ${BASE_ENV%%=*}
fi
