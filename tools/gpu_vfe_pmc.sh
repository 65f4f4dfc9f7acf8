# PMC passes over the PillarVFE kernel of the LiDAR step (one rocprofv3 run per pass, kernel filter).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6/vfe_pmc
cd /tmp && export TMPDIR=/tmp && cd $R
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU" \
            "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS SQ_INSTS_BRANCH" \
            "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  rm -rf /tmp/vpmc$i
  timeout -s KILL 150 rocprofv3 --pmc $pass --kernel-include-regex "pillar_vfe" --output-format csv -d /tmp/vpmc$i -o run -- python bench.py --only lidar --steps 2 --warmup 1 > gpurun_out/r6/vfe_pmc/p$i.log 2>&1 || { echo "PASS $i FAILED"; tail -5 gpurun_out/r6/vfe_pmc/p$i.log; exit 1; }
  f=$(find /tmp/vpmc$i -name "*counter_collection.csv" | head -1)
  cp $f gpurun_out/r6/vfe_pmc/p$i.csv
done
python tools/pmc_summary.py pillar_vfe gpurun_out/r6/vfe_pmc/p*.csv > gpurun_out/r6/vfe_pmc/summary.md 2>&1 || true; cat gpurun_out/r6/vfe_pmc/summary.md
echo VFE_PMC_OK
