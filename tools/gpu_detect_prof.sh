# Kernel traces of the camera-only bench, fused vs unfused Detect, on one box.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r4
cd /tmp && export TMPDIR=/tmp && cd $R
for mode in fused unfused; do
  F=""; [ $mode = unfused ] && F="--unfused-detect"
  rm -rf /tmp/dp_$mode
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/dp_$mode -o run -- python bench.py --only camera --steps 8 --warmup 3 $F > gpurun_out/r4/dp_$mode.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/r4/dp_$mode.log; exit 1; }
  tail -1 gpurun_out/r4/dp_$mode.log | cut -c1-200
  f=$(find /tmp/dp_$mode -name "*kernel_trace.csv" | head -1)
  python tools/step_stats.py $f --marker yolo_stem --steps 6 > gpurun_out/r4/step_stats_camera_$mode.txt && head -30 gpurun_out/r4/step_stats_camera_$mode.txt
done
