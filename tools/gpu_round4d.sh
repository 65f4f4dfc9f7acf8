# Round-4 GPU check, part 4: RCCL / hx3 / fp32-gate tests, LiDAR PMC passes (hx3 epilogue bank
# conflicts), a rocprofv3 kernel trace of the live-driver bench, the 1-GPU headline bench.
# A step that times out, aborts or segfaults ends the script (nothing more runs on the GPU).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4
mkdir -p $O
cd $R
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2: stopping"; exit $1;; esac; }
echo "== tests"
timeout -k 10 900 python -u -m pytest tests/test_rccl.py tests/test_hx3_gpu.py tests/test_fp32_mode_gpu.py \
  -v -s -m gpu --timeout 300 --timeout-method thread > $O/pytest_d.log 2>&1; rc=$?
grep -E 'PASSED|FAILED|ERROR' $O/pytest_d.log | tail -40; tail -2 $O/pytest_d.log
[ $rc -eq 0 ] || { echo TESTS_RC=$rc; grep -E '^E ' $O/pytest_d.log | head -30; }
fatal $rc pytest
echo "== headline bench"
timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 > $O/bench.json 2> $O/bench.err; rc=$?
[ $rc -eq 0 ] || { echo BENCH_FAILED; tail -20 $O/bench.err; }
fatal $rc bench
cat $O/bench.json
echo "== LiDAR PMC"
timeout -k 10 500 bash tools/gpu_lidar_pmc.sh; rc=$?
fatal $rc lidar_pmc
[ $rc -eq 0 ] && for k in "conv_hx3_kernel<8, 64" "conv_hx3_kernel<8, 128" "conv_hx3s2" "bev_neck" "pillar_vfe"; do
  echo "-- $k"; python tools/pmc_summary.py "$k" gpurun_out/pmc_lidar/p*.csv || true; done
echo "== driver bench kernel trace"
export PYTHONPATH=$R
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/drvprof -o drv -- python3 $R/tools/driver_bench.py \
  --camera 256 --lidar 256 --batch 32 --workers 3 > $O/drvprof_run.log 2>&1; rc=$?
cd $R
[ $rc -eq 0 ] || { echo PROF_FAILED; tail -20 $O/drvprof_run.log; }
fatal $rc drvprof
f=$(find $O/drvprof -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && head -40 "$f"
echo DONE
