# Round-4 GPU check, part 5: hx3 direct-epilogue twins (bit identity, per-layer timing) and the
# pipelined served batcher (served GPU tests, served bench shm / raw).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4
mkdir -p $O
cd $R
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2: stopping"; exit $1;; esac; }
echo "== tests"
timeout -k 10 600 python -u -m pytest tests/test_hx3_gpu.py tests/test_drivers_gpu.py -v -m gpu --timeout 300 \
  --timeout-method thread -k "direct or served" > $O/pytest_e.log 2>&1; rc=$?
grep -E 'PASSED|FAILED|ERROR' $O/pytest_e.log | tail -30; tail -2 $O/pytest_e.log
[ $rc -eq 0 ] || { echo TESTS_RC=$rc; grep -E '^E ' $O/pytest_e.log | head -30; }
fatal $rc pytest
echo "== hx3 tiles"
timeout -k 10 300 python -u tools/bench_conv_x3.py 0,111,112,115,116,151,152,155,156,121,122,123,124,161,162,163,164 \
  pp. --pair > $O/hx3_direct_tiles.jsonl 2>&1; rc=$?
grep layer $O/hx3_direct_tiles.jsonl || tail -20 $O/hx3_direct_tiles.jsonl
fatal $rc tiles
echo "== served"
NOTEST=1 SPROCS=1 timeout -k 10 600 bash tools/gpu_served3.sh; rc=$?
fatal $rc served
echo DONE
