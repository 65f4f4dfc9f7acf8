# Round 5: served raw / shm with 1, 2 and 4 server processes sharing the port (GIL-bound byte copies).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5
cd $R
for W in raw shm; do
  for S in ${SPS:-1 2 4}; do
    timeout -k 10 300 python tools/served_bench.py --frames 512 --window 8 --client-procs 4 --workers 32 --wire $W --server-procs $S \
      --json-out gpurun_out/r5/served_sp${S}_$W.json > gpurun_out/r5/served_sp${S}_$W.log 2>&1 || { echo BENCH_FAILED $W $S; tail -20 gpurun_out/r5/served_sp${S}_$W.log; exit 1; }
    python - gpurun_out/r5/served_sp${S}_$W.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[1], d["value"], d["server_requests_per_execution"], d["host_cpu_cores_busy"])
PY
  done
done
