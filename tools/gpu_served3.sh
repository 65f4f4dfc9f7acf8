# Served path, round 3: where the time goes (server stage clock) at P = 4 shm and P = 2 raw.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
P=${P:-4}
[ -n "$NOTEST" ] || timeout -k 10 400 python -u -m pytest tests/test_drivers_gpu.py tests/test_kserve.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/served3_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error" gpurun_out/served3_tests.log | tail -20; exit 1; }
[ -n "$NOTEST" ] || tail -1 gpurun_out/served3_tests.log
for W in ${WIRES:-shm raw}; do
  timeout -k 10 400 python tools/served_bench.py --frames 512 --window 8 --client-procs $P --workers ${WORKERS:-32} --server-procs ${SPROCS:-1} --wire $W --json-out gpurun_out/served3_p${P}_s${SPROCS:-1}${TAG}_$W.json --server-profile gpurun_out/served3_prof_p${P}_s${SPROCS:-1}${TAG}_$W.json > gpurun_out/served3_p${P}_s${SPROCS:-1}${TAG}_$W.log 2>&1 || { echo BENCH_FAILED $W; tail -20 gpurun_out/served3_p${P}_s${SPROCS:-1}${TAG}_$W.log; exit 1; }
  tail -1 gpurun_out/served3_p${P}_s${SPROCS:-1}${TAG}_$W.log | cut -c1-400
  cat gpurun_out/served3_prof_p${P}_s${SPROCS:-1}${TAG}_$W.json; echo
done
