# Same-box sweep of the step's existing switches: ROUNDS rounds, every config once per round in a rotated
# order, 30 timed steps each; tools/knob_table.py prints the per-config medians.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
TAG=${TAG:-knobs}
ROUNDS=${ROUNDS:-5}
mkdir -p gpurun_out/r6/$TAG
if [ "${SET:-1}" = "2" ]; then  # the follow-up on another box: the two candidates and both together
  CONFIGS=("default||" "neck2|TCA_NECK_VARIANT=2|" "vfelin2|TCA_VFE_LIN2=1|" "both|TCA_NECK_VARIANT=2 TCA_VFE_LIN2=1|")
elif [ "${SET:-1}" = "3" ]; then  # after both became the default: against the previous defaults
  CONFIGS=("default||" "r6start|TCA_NECK_VARIANT=0 TCA_VFE_LIN2=0|")
elif [ "${SET:-1}" = "5" ]; then  # the LiDAR software-pipeline split points
  CONFIGS=("default||" "pipe5||--lidar-pipeline 5" "pipe1||--lidar-pipeline 1" "lidar3||--only lidar"
           "lidar5||--only lidar --lidar-pipeline 5")
elif [ "${SET:-1}" = "6" ]; then  # mode 5 against mode 3 (the default) only
  CONFIGS=("default||" "pipe5||--lidar-pipeline 5")
elif [ "${SET:-1}" = "10" ]; then  # fewer workgroups for the neck (it runs beside the first down blocks in mode 5)
  CONFIGS=("default||" "neckg128|TCA_NECK_GRID=128|" "neckg160|TCA_NECK_GRID=160|" "neckg192|TCA_NECK_GRID=192|")
elif [ "${SET:-1}" = "11" ]; then  # the 3/4-CU neck grid (default) against the full grid
  CONFIGS=("default||" "neckfull|TCA_NECK_GRID=256|")
elif [ "${SET:-1}" = "12" ]; then  # the PillarVFE grid under mode 5 (it runs beside the down blocks)
  CONFIGS=("default||" "vfeg512|TCA_VFE_GRID=512|" "vfeg1024|TCA_VFE_GRID=1024|" "vfeg4096|TCA_VFE_GRID=4096|")
elif [ "${SET:-1}" = "13" ]; then  # per-point voxeliser passes over a bounded grid (TCA_VOX_GRID workgroups per frame)
  CONFIGS=("default||" "voxg8|TCA_VOX_GRID=8|" "voxg16|TCA_VOX_GRID=16|" "voxg32|TCA_VOX_GRID=32|" "voxg64|TCA_VOX_GRID=64|")
elif [ "${SET:-1}" = "14" ]; then  # the follow-up: the two best caps of set 13 against one chunk per workgroup
  CONFIGS=("default||" "voxg16|TCA_VOX_GRID=16|" "voxg32|TCA_VOX_GRID=32|")
elif [ "${SET:-1}" = "15" ]; then  # non-temporal loads of the streamed point data in the LiDAR front (TCA_VOX_NT)
  CONFIGS=("default||" "voxnt|TCA_VOX_NT=1|")
elif [ "${SET:-1}" = "16" ]; then  # mode 5: the next front waits for the first 1 / 2 down blocks (TCA_FRONT_AFTER)
  CONFIGS=("default||" "fa1|TCA_FRONT_AFTER=1|" "fa2|TCA_FRONT_AFTER=2|")
elif [ "${SET:-1}" = "17" ]; then  # after TCA_FRONT_AFTER=1 became the default: against 0 (the front right after the neck / NMS)
  CONFIGS=("default||" "fa0|TCA_FRONT_AFTER=0|")
elif [ "${SET:-1}" = "18" ]; then  # the front gate at conv granularity (default: after block 1 = 4 convs)
  CONFIGS=("default||" "fc2|TCA_FRONT_AFTER_CONVS=2|" "fc3|TCA_FRONT_AFTER_CONVS=3|" "fc5|TCA_FRONT_AFTER_CONVS=5|"
           "fc6|TCA_FRONT_AFTER_CONVS=6|")
elif [ "${SET:-1}" = "4" ]; then  # launch shapes and tiles (TCA_VFE_GRID, TCA_NECK_GRID, TCA_*_TILE)
  CONFIGS=("default||" "vfeg1024|TCA_VFE_GRID=1024|" "vfeg4096|TCA_VFE_GRID=4096|" "neckg192|TCA_NECK_GRID=192|"
           "neckg224|TCA_NECK_GRID=224|" "hx3t5|TCA_HX3_TILE=5|" "hx3t4|TCA_HX3_TILE=4|" "winot1|TCA_WINO_TILE=1|"
           "lazy0|TCA_LAZY_CANVAS=0|" "s2sp|TCA_S2SP=1|")
else
  CONFIGS=("default||" "neck1|TCA_NECK_VARIANT=1|" "neck2|TCA_NECK_VARIANT=2|" "pipe2||--lidar-pipeline 2"
           "pipe4||--lidar-pipeline 4" "wino64|TCA_WINO_MIN_N=64|" "vfelin2|TCA_VFE_LIN2=1|" "split||--graph-mode split")
fi
n=${#CONFIGS[@]}
for k in $(seq 1 $ROUNDS); do
  for i in $(seq 0 $((n - 1))); do
    c=${CONFIGS[$(( (i + k) % n ))]}
    name=${c%%|*}; rest=${c#*|}; envs=${rest%%|*}; flags=${rest#*|}
    env $envs timeout -k 10 300 python bench.py --steps 30 --warmup 5 $flags > gpurun_out/r6/$TAG/${name}_$k.log 2>&1 || { echo "BENCH_FAILED $name"; tail -20 gpurun_out/r6/$TAG/${name}_$k.log; exit 1; }
    echo "$name $k $(tail -1 gpurun_out/r6/$TAG/${name}_$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'])")"
  done
done
