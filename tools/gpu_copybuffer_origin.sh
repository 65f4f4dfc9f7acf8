# Round 6: where the served path's blit-kernel copies come from.  A 4 + 4 client shm run under a kernel +
# memory-copy + HIP API trace (no counters), then tools/copybuffer_origin.py joins every copyBuffer dispatch
# to the HIP call that issued it.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6/cbo
cd /tmp && export TMPDIR=/tmp
rm -rf /tmp/cbo
timeout -k 10 400 rocprofv3 --kernel-trace --memory-copy-trace --hip-runtime-trace --output-format csv -d /tmp/cbo \
  -o %pid% -- python3 $R/tools/served_bench.py --frames 128 --window 8 --client-procs 4 --workers 96 --wire ${WIRE:-shm} \
  --json-out $R/gpurun_out/r6/cbo/served_${WIRE:-shm}.json > $R/gpurun_out/r6/cbo/served.log 2>&1 || { echo FAILED; tail -30 $R/gpurun_out/r6/cbo/served.log; exit 1; }
tail -1 $R/gpurun_out/r6/cbo/served.log | cut -c1-300
d=$(dirname $(find /tmp/cbo -name "*_kernel_trace.csv" | head -1))
python3 $R/tools/copybuffer_origin.py $d > $R/gpurun_out/r6/cbo/origin_${WIRE:-shm}.txt || exit 1
head -30 $R/gpurun_out/r6/cbo/origin_${WIRE:-shm}.txt
for f in $d/*_memory_copy_trace.csv; do python3 - "$f" <<'PY'
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
c = collections.defaultdict(lambda: [0, 0, 0])
for r in rows:
    k = r.get("Direction", "?")
    c[k][0] += 1
    c[k][1] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    c[k][2] += int(r.get("Size", 0) or 0)
print(sys.argv[1].split("/")[-1], {k: (v[0], round(v[1] / 1e6, 2), round(v[2] / 2**20, 1)) for k, v in c.items()})
PY
done > $R/gpurun_out/r6/cbo/copies_${WIRE:-shm}.txt
cat $R/gpurun_out/r6/cbo/copies_${WIRE:-shm}.txt
