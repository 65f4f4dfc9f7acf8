# bench launch contract on a 1-GPU box: default run, --gpus 2 refusal, gloo 2-rank self-launch, RCCL tests.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 120 python -u -m pytest tests/test_rccl.py -v -m gpu --timeout 60 --timeout-method thread > gpurun_out/rccl_tests.log 2>&1 || { echo RCCL_TESTS_FAILED; tail -30 gpurun_out/rccl_tests.log; }
tail -4 gpurun_out/rccl_tests.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_default.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log | cut -c1-600
timeout -k 10 120 python bench.py --gpus 2 --steps 5 --warmup 2 > gpurun_out/bench_gpus2_refuse.log 2>&1 && { echo "GPUS2 DID NOT REFUSE"; exit 1; }
tail -2 gpurun_out/bench_gpus2_refuse.log
TCA_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 5 --warmup 2 --batch 8 > gpurun_out/bench_gloo2.log 2>&1 || { echo GLOO2_FAILED; tail -20 gpurun_out/bench_gloo2.log; exit 1; }
grep '^{' gpurun_out/bench_gloo2.log | cut -c1-300
