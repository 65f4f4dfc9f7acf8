# Round-4 GPU check, part 3: RCCL two-graph arrangements, driver bench (1 GPU, 2 gloo ranks), layer tables.
# A step that times out, aborts or segfaults ends the script (nothing more runs on the GPU).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4
mkdir -p $O
cd $R
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2: stopping"; exit $1;; esac; }
for v in two_comms one_comm_prewarm one_comm; do
  echo "== rccl $v"
  timeout -k 5 90 python -u tools/rccl_two_graphs.py --variant $v > $O/rccl_$v.log 2>&1; rc=$?
  grep -v "^RCCL\|^HIP\|^ROCm\|^Hostname\|^Librccl" $O/rccl_$v.log | tail -30
  fatal $rc rccl_$v
  grep -q "^Timeout" $O/rccl_$v.log && { echo "rccl_$v hung (faulthandler): stopping"; exit 1; }
done
echo "== driver bench"
timeout -k 10 300 python -u tools/driver_bench.py --camera 1024 --lidar 1024 --batch 32 --workers 3 \
  > $O/driver_bench.json 2> $O/driver_bench.err; rc=$?
[ $rc -eq 0 ] || { echo DRIVER_BENCH_FAILED; tail -30 $O/driver_bench.err; }
fatal $rc driver_bench
cat $O/driver_bench.json
echo "== driver bench, 2 ranks on the one card (gloo rehearsal)"
TCA_DIST_BACKEND=gloo timeout -k 10 300 python -u tools/driver_bench.py --gpus 2 --camera 256 --lidar 256 --batch 32 \
  --workers 2 > $O/driver_bench_dp2.log 2>&1; rc=$?
grep -v Gloo $O/driver_bench_dp2.log | tail -5
fatal $rc driver_bench_dp2
echo "== layers"
for br in camera lidar; do
  timeout -k 10 240 python -u tools/layer_times.py --branch $br > $O/layers_$br.json 2> $O/layers_$br.txt; rc=$?
  [ $rc -eq 0 ] || { echo LAYERS_FAILED $br; tail -20 $O/layers_$br.txt; }
  fatal $rc layers_$br
  head -30 $O/layers_$br.txt
done
