set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $R && timeout -k 10 400 rocprofv3 --kernel-trace -d /tmp/second_prof -o run -- python tools/second_probe.py > gpurun_out/second_prof.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/second_prof.log; exit 1; }
python tools/rocpd_stats.py /tmp/second_prof/run_results.db --top 70 > gpurun_out/second_kernel_stats.txt && cat gpurun_out/second_kernel_stats.txt | cut -c1-150
