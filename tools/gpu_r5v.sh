# Round 5: served path after the decode-only YOLO kernel (4 + 4 clients, shm and raw).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5
cd $R
for W in shm raw; do
  timeout -k 10 300 python tools/served_bench.py --frames 512 --window 8 --client-procs 4 --workers 32 --wire $W \
    --json-out gpurun_out/r5/served_dec_$W.json --server-profile gpurun_out/r5/served_prof_dec_$W.json \
    > gpurun_out/r5/served_dec_$W.log 2>&1 || { echo BENCH_FAILED $W; tail -20 gpurun_out/r5/served_dec_$W.log; exit 1; }
  python - gpurun_out/r5/served_dec_$W.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[1], d["value"], d["server_requests_per_execution"], d["client_ms_per_frame"])
PY
done
