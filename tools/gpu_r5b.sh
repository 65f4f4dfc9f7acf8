# Round 5: the remote (KServe client) driver path on the device: driver_bench --engine remote at the
# reference's defaults (one message per callback, sync RPC) and batched (async, 3 workers), plus a
# rocprofv3 kernel trace of the default-flags run.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r5
cd $R
timeout -k 10 400 python tools/driver_bench.py --engine remote --camera 256 --lidar 256 --batch 1 --workers 1 > gpurun_out/r5/driver_remote_b1.log 2>&1 || { echo DRV1_FAILED; tail -30 gpurun_out/r5/driver_remote_b1.log; exit 1; }
tail -1 gpurun_out/r5/driver_remote_b1.log | cut -c1-600
timeout -k 10 400 python tools/driver_bench.py --engine remote --mode async --camera 512 --lidar 512 --batch 32 --workers 3 > gpurun_out/r5/driver_remote_b32.log 2>&1 || { echo DRV32_FAILED; tail -30 gpurun_out/r5/driver_remote_b32.log; exit 1; }
tail -1 gpurun_out/r5/driver_remote_b32.log | cut -c1-600
cd /tmp && export TMPDIR=/tmp && cd $R
rm -rf /tmp/rk
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/rk -o run -- python tools/driver_bench.py --engine remote --camera 64 --lidar 64 --batch 1 --workers 1 > gpurun_out/r5/driver_remote_prof.log 2>&1 || { echo PROF_FAILED; tail -30 gpurun_out/r5/driver_remote_prof.log; exit 1; }
f=$(find /tmp/rk -name "*kernel_stats.csv" | head -1)
cp $f gpurun_out/r5/driver_remote_kernel_stats.csv
python - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r5/driver_remote_kernel_stats.csv")))
for r in sorted(rows, key=lambda r: -float(r.get("TotalDurationNs", 0)))[:60]:
    print(r.get("Calls"), r.get("TotalDurationNs"), r["Name"][:110])
PY
