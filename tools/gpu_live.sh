# Live-driver device path on one GPU: its GPU tests, then tools/driver_bench.py.
#   usage: bash tools/gpu_live.sh [extra pytest paths...]   env PROF=1 adds a rocprofv3 kernel trace of the bench
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/live
cd $R
O=gpurun_out/live
timeout -k 10 600 python -u -m pytest tests/test_live.py tests/test_draw.py "$@" -x -v -m gpu --timeout 300 \
  --timeout-method thread > $O/pytest.log 2>&1 || { echo TESTS_FAILED; tail -40 $O/pytest.log; exit 1; }
grep -cE 'PASSED' $O/pytest.log; tail -1 $O/pytest.log
timeout -k 10 300 python -u tools/driver_bench.py --camera 1024 --lidar 1024 --batch 32 --workers ${WORKERS:-3} \
  > $O/driver_bench.json 2> $O/driver_bench.err || { echo DRIVER_BENCH_FAILED; tail -30 $O/driver_bench.err; exit 1; }
cat $O/driver_bench.json
if [ -n "$PROF" ]; then
  cd /tmp && export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof -o drv -- python3 $R/tools/driver_bench.py \
    --camera 256 --lidar 256 --batch 32 --workers ${WORKERS:-3} > $R/$O/prof_run.log 2>&1 || { echo PROF_FAILED; tail -20 $R/$O/prof_run.log; exit 1; }
  echo PROF_OK
fi
