# Round 6: one server process for both models vs one server process per model (--model-procs), 4 + 4
# client processes, window 16, 96 server threads per process, devshm and shm, two rounds in rotated order.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
OUT=gpurun_out/r6/served_split
mkdir -p $OUT
for k in 1 2; do
  for W in devshm shm; do
    for T in one split; do
      if [ $k = 2 ]; then T=$([ $T = one ] && echo split || echo one); fi
      F=$([ $T = split ] && echo --model-procs || echo)
      timeout -k 10 300 python tools/served_bench.py --frames 1024 --window 16 --client-procs 4 --workers 96 --wire $W $F --json-out $OUT/${W}_${T}_$k.json > $OUT/${W}_${T}_$k.log 2>&1 || { echo FAILED $W $T; tail -20 $OUT/${W}_${T}_$k.log; exit 1; }
      echo "$W $T $k: $(python3 -c "import json; d=json.load(open('$OUT/${W}_${T}_$k.json')); print(d['value'], d['server_requests_per_execution'], d['host_cpu_cores_busy'])")"
    done
  done
done
