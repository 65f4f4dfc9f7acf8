# PMC passes for the fp32 fused neck (tools/bench_neck.py variant 3 at batch 32), each pass its own run.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd $R
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU" \
            "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM" \
            "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  rm -rf /tmp/npmc$i
  timeout -s KILL 120 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d /tmp/npmc$i -o run -- python tools/bench_neck.py 32 0 > gpurun_out/pmc/neck_p$i.log 2>&1 || { echo "PASS $i FAILED"; tail -5 gpurun_out/pmc/neck_p$i.log; exit 1; }
  f=$(find /tmp/npmc$i -name "*counter_collection.csv" | head -1)
  cp $f gpurun_out/pmc/neck_r5_p$i.csv
done
python tools/pmc_summary.py bev_neck_head_x3 gpurun_out/pmc/neck_r5_p*.csv > gpurun_out/pmc_neck_r5.md && tail -6 gpurun_out/pmc_neck_r5.md
