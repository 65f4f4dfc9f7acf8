# Multi-rank rehearsal of bench.py (and, with DRIVERS=1, of the data-parallel live drivers) on ONE
# GPU: ranks share the card over host-staged gloo (TCA_DIST_BACKEND=gloo; RCCL refuses two ranks on
# one device).  Exercises the N>1 logic (pre-flight, calibration broadcast, gathers, barrier,
# max-reduce, JSON line; the drivers' host ring) except RCCL itself.
#   CFGS: "ranks ingest" pairs (default "2 local" "2 rccl" "4 local" "8 local")
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/dp
cd $R
export TCA_DIST_BACKEND=gloo
CFGS=${CFGS:-"2_local 2_rccl 4_local 8_local"}
for cfg in $CFGS; do
  n=${cfg%_*}; ing=${cfg#*_}
  timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus $n --steps 5 --warmup 2 --ingest $ing > gpurun_out/dp/dp_rehearsal_${n}_${ing}.log 2>&1 || { echo FAILED $n $ing; tail -30 gpurun_out/dp/dp_rehearsal_${n}_${ing}.log; exit 1; }
  grep '^{' gpurun_out/dp/dp_rehearsal_${n}_${ing}.log > gpurun_out/dp/dp_rehearsal_${n}_${ing}.json
  echo "n=$n ingest=$ing: $(cut -c1-200 gpurun_out/dp/dp_rehearsal_${n}_${ing}.json)"
done
if [ -n "$DRIVERS" ]; then
  timeout -k 10 500 python tools/driver_bench.py --gpus ${DRIVER_GPUS:-8} --camera 256 --lidar 256 --batch 16 > gpurun_out/dp/driver_dp_${DRIVER_GPUS:-8}.log 2>&1 || { echo DRIVERS_FAILED; tail -30 gpurun_out/dp/driver_dp_${DRIVER_GPUS:-8}.log; exit 1; }
  grep '^{' gpurun_out/dp/driver_dp_${DRIVER_GPUS:-8}.log | tail -1 > gpurun_out/dp/driver_dp_${DRIVER_GPUS:-8}.json
  cut -c1-300 gpurun_out/dp/driver_dp_${DRIVER_GPUS:-8}.json
fi
