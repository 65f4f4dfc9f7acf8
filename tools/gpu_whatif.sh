# What-if bounds of the headline (tools/whatif_bench.py, diagnostic only): each WHATIF mode against the
# unchanged step, ROUNDS alternating rounds.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
TAG=${TAG:-whatif}
mkdir -p gpurun_out/r6/$TAG
for k in $(seq 1 ${ROUNDS:-3}); do
  for m in none ${MODES:-nopost noneck novox}; do
    if [ $m = none ]; then unset WHATIF; else export WHATIF=$m; fi
    timeout -k 10 300 python tools/whatif_bench.py --steps 30 --warmup 5 > gpurun_out/r6/$TAG/${m}_$k.log 2>&1 || { echo "FAILED $m"; tail -20 gpurun_out/r6/$TAG/${m}_$k.log; exit 1; }
    echo "$m $k $(tail -1 gpurun_out/r6/$TAG/${m}_$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'])")"
  done
done
unset WHATIF
