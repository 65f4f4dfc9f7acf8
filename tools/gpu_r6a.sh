set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/r6
timeout -k 10 600 python -u -m pytest tests/test_remote_device_gpu.py tests/test_numa_gpu.py tests/test_detect_fused_gpu.py -x -v -s -m gpu --timeout 300 --timeout-method thread > gpurun_out/r6/pytest_a.log 2>&1 || { echo TESTS_FAILED; grep -E 'FAILED|Error' gpurun_out/r6/pytest_a.log | tail -20; tail -40 gpurun_out/r6/pytest_a.log; exit 1; }
tail -1 gpurun_out/r6/pytest_a.log
timeout -k 10 120 python tools/copy_path_probe.py > gpurun_out/r6/copy_probe.log 2>&1 || { echo PROBE_FAILED; tail -20 gpurun_out/r6/copy_probe.log; exit 1; }
tail -1 gpurun_out/r6/copy_probe.log
cd /tmp && export TMPDIR=/tmp && cd $R
rm -rf /tmp/cp
timeout -k 10 120 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d /tmp/cp -o run -- python tools/copy_path_probe.py > gpurun_out/r6/copy_probe_prof.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/r6/copy_probe_prof.log; exit 1; }
for f in $(find /tmp/cp -name "*stats.csv"); do cp $f gpurun_out/r6/copyprobe_$(basename $f); done
WIRES="raw devshm" bash tools/gpu_r6_remote.sh
