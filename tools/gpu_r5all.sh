# Round 5 combined GPU session: neck checks + step profile, remote-client tests + NUMA + fan-out + timeline,
# remote driver bench.  Each part stops the call on failure.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_neck_r5.sh > gpurun_out/r5/part_neck.txt 2>&1 || { echo NECK_PART_FAILED; tail -30 gpurun_out/r5/part_neck.txt; exit 1; }
cat gpurun_out/r5/part_neck.txt | cut -c1-300
bash tools/gpu_r5a.sh > gpurun_out/r5/part_a.txt 2>&1 || { echo A_PART_FAILED; tail -30 gpurun_out/r5/part_a.txt; exit 1; }
cat gpurun_out/r5/part_a.txt | cut -c1-300
bash tools/gpu_r5b.sh > gpurun_out/r5/part_b.txt 2>&1 || { echo B_PART_FAILED; tail -30 gpurun_out/r5/part_b.txt; exit 1; }
cat gpurun_out/r5/part_b.txt | cut -c1-400 | head -40
