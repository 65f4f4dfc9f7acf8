# End of round 4: headline kernel profile (per-kernel stats per step) and five back-to-back headline runs.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r4
cd $R
TAG=r4final bash tools/gpu_step_profile.sh > gpurun_out/r4/final_step_profile.txt 2>&1 || { echo STEP_PROFILE_FAILED; tail -20 gpurun_out/r4/final_step_profile.txt; exit 1; }
head -3 gpurun_out/r4/final_step_profile.txt | cut -c1-200
for i in 1 2 3 4 5; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 10 > gpurun_out/r4/final_rep_$i.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/r4/final_rep_$i.log; exit 1; }
  echo "rep $i $(tail -1 gpurun_out/r4/final_rep_$i.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
