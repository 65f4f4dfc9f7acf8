# One PMC pass over the LiDAR and the camera step: scalar vs vector instruction mix per kernel
# (tools/salu_table.py).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6/salu
cd /tmp && export TMPDIR=/tmp && cd $R
for br in lidar camera; do
  rm -rf /tmp/salu_$br
  timeout -s KILL 150 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d /tmp/salu_$br -o run -- python bench.py --only $br --steps 2 --warmup 1 > gpurun_out/r6/salu/$br.log 2>&1 || { echo "SALU $br FAILED"; tail -5 gpurun_out/r6/salu/$br.log; exit 1; }
  f=$(find /tmp/salu_$br -name "*counter_collection.csv" | head -1)
  cp $f gpurun_out/r6/salu/${br}_counters.csv
  python tools/salu_table.py $f > gpurun_out/r6/salu/salu_$br.md || exit 1
  head -24 gpurun_out/r6/salu/salu_$br.md
done
