# Per-family 1-GPU numbers at an explicit batch (README "Other model families").
#   usage: BATCH=16 bash tools/gpu_families.sh
set -o pipefail
B=${BATCH:-16}
mkdir -p gpurun_out
run() { tag=$1; shift; timeout -k 10 300 python bench.py --batch $B --steps 30 --warmup 5 "$@" > gpurun_out/fam_${tag}_b$B.log 2>&1 || { echo FAILED $tag; tail -20 gpurun_out/fam_${tag}_b$B.log; exit 1; }; tail -1 gpurun_out/fam_${tag}_b$B.log | cut -c1-160; }
run second --only lidar --lidar-model second_iou
run centerpoint --only lidar --lidar-model centerpoint
run retinanet --only camera --camera-model retinanet
run fcos --only camera --camera-model fcos
run yolov4 --only camera --camera-model yolov4
