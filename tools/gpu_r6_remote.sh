# Round 6: the remote (KServe client) driver path over each wire at the reference's defaults (one
# message per callback, sync RPC): raw vs shm vs devshm, plus a rocprofv3 kernel trace of the devshm run.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r6/remote
cd $R
for w in ${WIRES:-raw devshm shm}; do
  timeout -k 10 400 python tools/driver_bench.py --engine remote --wire $w --camera 256 --lidar 256 --batch 1 --workers 1 > gpurun_out/r6/remote/driver_remote_b1_$w.log 2>&1 || { echo DRV_FAILED $w; tail -30 gpurun_out/r6/remote/driver_remote_b1_$w.log; exit 1; }
  tail -1 gpurun_out/r6/remote/driver_remote_b1_$w.log | cut -c1-400
done
cd /tmp && export TMPDIR=/tmp && cd $R
rm -rf /tmp/rk
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/rk -o run -- python tools/driver_bench.py --engine remote --wire devshm --camera 64 --lidar 64 --batch 1 --workers 1 > gpurun_out/r6/remote/driver_devshm_prof.log 2>&1 || { echo PROF_FAILED; tail -30 gpurun_out/r6/remote/driver_devshm_prof.log; exit 1; }
f=$(find /tmp/rk -name "*kernel_stats.csv" | head -1)
cp $f gpurun_out/r6/remote/driver_devshm_kernel_stats.csv
