# Round 5: remote driver bench, fan-out with / without streaming stores, served path (shm + raw, 1 and 2 server procs).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5
cd $R
bash tools/gpu_r5b.sh > gpurun_out/r5/part_b.txt 2>&1 || { echo B_PART_FAILED; tail -30 gpurun_out/r5/part_b.txt; exit 1; }
cat gpurun_out/r5/part_b.txt | cut -c1-600 | head -50
timeout -k 10 300 python tools/fanout_bench.py --threads 8,16,32 --json gpurun_out/r5/fanout_nt.json > gpurun_out/r5/fanout_nt.log 2>&1 || { echo FANOUT_FAILED; tail -10 gpurun_out/r5/fanout_nt.log; exit 1; }
TCA_HOST_COPY_NT=0 timeout -k 10 300 python tools/fanout_bench.py --threads 8,16,32 --json gpurun_out/r5/fanout_memcpy.json > gpurun_out/r5/fanout_memcpy.log 2>&1 || { echo FANOUT_FAILED; tail -10 gpurun_out/r5/fanout_memcpy.log; exit 1; }
tail -1 gpurun_out/r5/fanout_nt.log; tail -1 gpurun_out/r5/fanout_memcpy.log
for S in 1 2; do
  WIRES="shm raw" SPROCS=$S NOTEST=1 TAG=_r5 bash tools/gpu_served3.sh > gpurun_out/r5/served_s$S.txt 2>&1 || { echo SERVED_FAILED; tail -20 gpurun_out/r5/served_s$S.txt; exit 1; }
  grep -v '^{"wall_s"' gpurun_out/r5/served_s$S.txt | cut -c1-400
done
