# Served path, round 5: server worker threads vs requests in flight (4 + 4 clients x window 8 = 64),
# and GPU hardware queues per client process.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5
cd $R
run() {  # tag wire workers hwq
  timeout -k 10 300 python tools/served_bench.py --frames 512 --window 8 --client-procs 4 --workers $3 --wire $2 \
    --client-hw-queues $4 --json-out gpurun_out/r5/served_$1.json --server-profile gpurun_out/r5/served_prof_$1.json \
    > gpurun_out/r5/served_$1.log 2>&1 || { echo BENCH_FAILED $1; tail -20 gpurun_out/r5/served_$1.log; return 1; }
  python - gpurun_out/r5/served_$1.json <<'EOF'
import json, sys
d = json.load(open(sys.argv[1]))
print(sys.argv[1], d["value"], d["server_requests_per_execution"], d["host_cpu_cores_busy"], d["client_ms_per_frame"])
EOF
}
run w32_shm shm 32 0 &&
run w96_shm shm 96 0 &&
run w96q1_shm shm 96 1 &&
run w160q1_shm shm 160 1 &&
run w96q1_raw raw 96 1
