# Plain-fp32 hx twins: whole GPU suite + smoke + headline bench (round check), then the fp32 family benches.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_round_check2.sh || exit 1
for fam in "--only lidar --lidar-model centerpoint" "--only lidar --lidar-model second_iou" "--only camera --camera-model retinanet" "--only camera --camera-model fcos"; do
  tag=$(echo $fam | awk '{print $NF}')
  timeout -k 10 300 python bench.py $fam --batch 16 --steps 20 --warmup 5 > gpurun_out/fam_$tag.log 2>&1 || { echo BENCH_FAILED $tag; tail -20 gpurun_out/fam_$tag.log; exit 1; }
  echo "$tag $(tail -1 gpurun_out/fam_$tag.log | grep -o '"value": [0-9.]*')"
done
