# Round 6: copy paths per source kind (tools/copy_path_probe.py: timings + the device events torch.profiler
# records for each kind, blit kernel or DMA copy), no external tracer.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/r6
timeout -k 10 180 python tools/copy_path_probe.py > gpurun_out/r6/copy_probe_events.log 2>&1 || { echo PROBE_FAILED; tail -20 gpurun_out/r6/copy_probe_events.log; exit 1; }
tail -1 gpurun_out/r6/copy_probe_events.log | cut -c1-2000
