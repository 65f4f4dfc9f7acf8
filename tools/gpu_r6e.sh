# Round 6: copy paths (tools/copy_path_probe.py) under a kernel + memory-copy trace, and the remote
# driver over raw / devshm / shm at the reference's defaults (tools/gpu_r6_remote.sh).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6
cd $R
cd /tmp && export TMPDIR=/tmp && cd $R
rm -rf /tmp/cp
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d /tmp/cp -o run -- python tools/copy_path_probe.py > gpurun_out/r6/copy_probe_prof.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/r6/copy_probe_prof.log; exit 1; }
tail -1 gpurun_out/r6/copy_probe_prof.log
for f in $(find /tmp/cp -name "*.csv"); do cp $f gpurun_out/r6/copyprobe_$(basename $f); done
bash tools/gpu_r6_remote.sh
