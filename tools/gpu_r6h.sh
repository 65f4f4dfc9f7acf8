# Round 6: the camera's conv_xb layers (YOLOv5n b3 / b5 / b7, SPPF, PAN downsamples, unfused C3 convs):
# every fp32-mode tile per layer at batch 32 (tools/bench_conv_x3.py), then the remote wires bench.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6
cd $R
timeout -k 10 500 python tools/bench_conv_x3.py 0,80,81,82,83,84,85,86,87,60,1,2,5,6,20,22,24,25,26,27,41,42,47 y.b3,y.b5,y.b7,y.sp,y.h19,y.h22,y.c3c,y.c3d > gpurun_out/r6/camera_conv_tiles.jsonl 2> gpurun_out/r6/camera_conv_tiles.err || { echo TILES_FAILED; tail -20 gpurun_out/r6/camera_conv_tiles.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/r6/camera_conv_tiles.jsonl'):
    d = json.loads(l); print(d['layer'], 'auto', d['us_by_tile'].get('0'), 'best', d.get('best_tile'), d.get('best_us'))
"
