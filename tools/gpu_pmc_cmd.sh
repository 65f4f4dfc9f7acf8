# PMC passes (one rocprofv3 run per counter group) over an arbitrary command: CMD (python args), TAG
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd $R
TAG=${TAG:-cmd}
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU" \
            "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM" \
            "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE" \
            "TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  rm -rf /tmp/pmc$i
  timeout -s KILL 120 rocprofv3 --pmc $pass --output-format csv -d /tmp/pmc$i -o run -- python $CMD > gpurun_out/pmc/${TAG}_p$i.log 2>&1 || { echo "PASS $i FAILED"; tail -5 gpurun_out/pmc/${TAG}_p$i.log; exit 1; }
  f=$(find /tmp/pmc$i -name "*counter_collection.csv" | head -1)
  cp $f gpurun_out/pmc/${TAG}_p$i.csv
done
echo PMC_OK
