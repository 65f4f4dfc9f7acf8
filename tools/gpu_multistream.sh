set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
run() {
timeout -k 10 300 python bench.py --steps 40 --warmup 5 "$@" > gpurun_out/ms.log 2>&1 || { echo BENCH_FAILED "$@"; tail -30 gpurun_out/ms.log; exit 1; }
echo "$@" $(tail -1 gpurun_out/ms.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")
}
for i in 1 2; do
run --graph-mode fork
run --graph-mode split
run --graph-mode split --lidar-priority 1
run --graph-mode fork --lidar-priority 1
done
