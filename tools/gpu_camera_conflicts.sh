# Round 5: stem LDS write order (conflicts): tests + camera PMC conflicts for the stem.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5 $R/gpurun_out/pmc
cd $R
timeout -k 10 300 python -u -m pytest tests/test_stem_fused_gpu.py tests/test_c3_fused_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r5/stem_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/r5/stem_tests.log; exit 1; }
tail -1 gpurun_out/r5/stem_tests.log
cd /tmp && export TMPDIR=/tmp && cd $R
rm -rf /tmp/cpmc
timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVES GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d /tmp/cpmc -o run -- python bench.py --only camera --steps 3 --warmup 2 > gpurun_out/pmc/cam_conf.log 2>&1 || { echo PMC_FAILED; tail -5 gpurun_out/pmc/cam_conf.log; exit 1; }
f=$(find /tmp/cpmc -name "*counter_collection.csv" | head -1)
cp $f gpurun_out/pmc/cam_conf.csv
python - <<'PY'
import csv, collections
v = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open("gpurun_out/pmc/cam_conf.csv")):
    v[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in sorted(v.items(), key=lambda kv: -sum(kv[1]["SQ_LDS_BANK_CONFLICT"]) / max(1, len(kv[1]["SQ_LDS_BANK_CONFLICT"]))):
    c = d["SQ_LDS_BANK_CONFLICT"]; i = d["SQ_INSTS_LDS"]
    if c: print("%-60s conflicts/dispatch %12.0f  lds insts %12.0f" % (k, sum(c) / len(c), sum(i) / max(1, len(i))))
PY
