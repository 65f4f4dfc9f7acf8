# PMC passes for conv_wino.hip (tools/bench_wino.py, one shape / tile), each pass its own run.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp && cd $R
S=${SHAPE:-1}; T=${TILE:-132}
i=0
for pass in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU" \
            "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM" \
            "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  rm -rf /tmp/wpmc$i
  F32=${F32:-} SHAPE=$S TILES=$T timeout -s KILL 120 rocprofv3 --pmc $pass --kernel-trace --output-format csv -d /tmp/wpmc$i -o run -- python tools/bench_wino.py > gpurun_out/pmc/wino_p$i.log 2>&1 || { echo "PASS $i FAILED"; tail -5 gpurun_out/pmc/wino_p$i.log; exit 1; }
  f=$(find /tmp/wpmc$i -name "*counter_collection.csv" | head -1)
  cp $f gpurun_out/pmc/wino_s${S}_t${T}_p$i.csv
done
python tools/pmc_summary.py conv_wino_kernel gpurun_out/pmc/wino_s${S}_t${T}_p*.csv > gpurun_out/pmc_wino_s${S}_t${T}.md && tail -6 gpurun_out/pmc_wino_s${S}_t${T}.md
