# Round 6: served-path frame pairs/s against the client request window (8 / 16 / 32 in flight per client) over
# devshm and shm, 4 + 4 client processes, 96 server threads.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/r6/servedw
for W in devshm shm; do
  for win in 8 16 32; do
    timeout -k 10 300 python tools/served_bench.py --frames 1024 --window $win --client-procs 4 --workers 96 --wire $W --json-out gpurun_out/r6/servedw/served_${W}_w$win.json > gpurun_out/r6/servedw/served_${W}_w$win.log 2>&1 || { echo FAILED $W $win; tail -20 gpurun_out/r6/servedw/served_${W}_w$win.log; exit 1; }
    echo "$W window $win: $(python3 -c "import json; d=json.load(open('gpurun_out/r6/servedw/served_${W}_w$win.json')); print(d['value'], d.get('server_requests_per_execution'))")"
  done
done
