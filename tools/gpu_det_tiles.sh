# fp32 tile sweep on the YOLOv5n Detect head 1x1 convs (batch 32).
set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python tools/bench_conv_x3.py 0,80,81,82,83,84,85,86,87,1,2,5 y.det > gpurun_out/det_tiles.jsonl 2>&1 || { echo FAILED; tail -20 gpurun_out/det_tiles.jsonl; exit 1; }
cat gpurun_out/det_tiles.jsonl | cut -c1-400
