# Headline kernel profile (rocprofv3 kernel trace -> per-kernel stats, per step).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $R && timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/final_prof -o run -- python bench.py --steps 20 --warmup 5 > gpurun_out/final_prof.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/final_prof.log; exit 1; }
python tools/rocpd_stats.py /tmp/final_prof/run_results.db --top 45 --per-step 25 > gpurun_out/final_kernel_stats.txt && head -50 gpurun_out/final_kernel_stats.txt | cut -c1-160
