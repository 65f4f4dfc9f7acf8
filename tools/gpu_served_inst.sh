# Served path with model instances (TCA_SERVE_INSTANCES): served GPU tests, then the 4+4 client
# served bench per wire at 2 instances and (A/B) at 1.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
P=${P:-4}
[ -n "$NOTEST" ] || timeout -k 10 400 python -u -m pytest tests/test_drivers_gpu.py tests/test_kserve.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/inst_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error" gpurun_out/inst_tests.log | tail -20; exit 1; }
[ -n "$NOTEST" ] || tail -1 gpurun_out/inst_tests.log
for I in ${INSTS:-2 1}; do
  for W in ${WIRES:-devshm shm raw}; do
    TCA_SERVE_INSTANCES=$I timeout -k 10 400 python tools/served_bench.py --frames 512 --window 8 --client-procs $P --workers ${WORKERS:-32} --wire $W --json-out gpurun_out/inst${I}_p${P}_$W.json > gpurun_out/inst${I}_p${P}_$W.log 2>&1 || { echo BENCH_FAILED $I $W; tail -20 gpurun_out/inst${I}_p${P}_$W.log; exit 1; }
    echo "instances=$I wire=$W $(python -c "import json;d=json.load(open('gpurun_out/inst${I}_p${P}_$W.json'));print(d['value'], d.get('server_requests_per_execution'))")"
  done
done
