# Round 6: copy paths (tools/copy_path_probe.py) under a kernel + memory-copy trace, and the remote
# driver over raw / devshm / shm at the reference's defaults (tools/gpu_r6_remote.sh).  The probe has
# crashed at interpreter exit under the tracer (after its measurements): the trace is kept either way.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6
cd $R
cd /tmp && export TMPDIR=/tmp && cd $R
rm -rf /tmp/cp
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d /tmp/cp -o run -- python tools/copy_path_probe.py > gpurun_out/r6/copy_probe_prof.log 2>&1
rc=$?
echo "probe under rocprofv3: rc=$rc"
case $rc in 124|137) exit $rc ;; esac
for f in $(find /tmp/cp -name "*.csv"); do cp $f gpurun_out/r6/copyprobe_$(basename $f); done
ls gpurun_out/r6 | grep copyprobe
bash tools/gpu_r6_remote.sh
