# Multi-rank rehearsal of bench.py on ONE GPU: ranks share the card over host-staged gloo
# (TCA_DIST_BACKEND=gloo; RCCL refuses two ranks on one device).  Exercises the N>1 bench
# logic (calibration broadcast, gathers, barrier, max-reduce, JSON line) except RCCL itself.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
export TCA_DIST_BACKEND=gloo
for cfg in "2 local" "2 rccl" "4 local"; do
  set -- $cfg
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $1 --master-addr 127.0.0.1 --master-port 29611 bench.py --gpus $1 --steps 5 --warmup 2 --ingest $2 > gpurun_out/dp_rehearsal_$1_$2.log 2>&1 || { echo FAILED $1 $2; tail -30 gpurun_out/dp_rehearsal_$1_$2.log; exit 1; }
  echo "n=$1 ingest=$2: $(grep '^{' gpurun_out/dp_rehearsal_$1_$2.log | cut -c1-220)"
done
