# wx3 ablations (TCA_WX3_DBG bits: 1 no transform, 2 no raw loads, 4 no epilogue stores, 8 no step barrier)
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
for d in ${DBGS:-0 3 4 15 31}; do
  TCA_WX3_DBG=$d timeout -k 10 120 python -u tools/bench_conv_x3.py 132 pp.b2.conv --pair > gpurun_out/wx3_abl_$d.jsonl 2>&1 || { echo ABL_FAILED $d; tail -5 gpurun_out/wx3_abl_$d.jsonl; exit 1; }
  echo "dbg=$d $(grep -o '"us_by_tile": {[^}]*}' gpurun_out/wx3_abl_$d.jsonl)"
done
