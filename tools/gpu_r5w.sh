# Round 5: served path with bulk gRPC transport options (16 MB HTTP/2 frames, large TCP reads) vs defaults.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5
cd $R
for W in raw shm; do
  for B in 1 0; do
    TCA_GRPC_BULK=$B timeout -k 10 300 python tools/served_bench.py --frames 512 --window 8 --client-procs 4 --workers 32 --wire $W \
      --json-out gpurun_out/r5/served_bulk${B}_$W.json > gpurun_out/r5/served_bulk${B}_$W.log 2>&1 || { echo BENCH_FAILED $W $B; tail -20 gpurun_out/r5/served_bulk${B}_$W.log; exit 1; }
    python - gpurun_out/r5/served_bulk${B}_$W.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[1], d["value"], d["server_requests_per_execution"], d["client_ms_per_frame"]["camera"])
PY
  done
done
