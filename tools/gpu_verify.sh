# GPU verification of HEAD: gpu tests, headline bench, kernel stats profile.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/verify_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/verify_tests.log; exit 1; }
timeout -k 10 300 python bench.py --steps 50 --warmup 5 > gpurun_out/verify_bench.log 2>&1 || { echo BENCH_FAILED; tail -30 gpurun_out/verify_bench.log; exit 1; }
tail -1 gpurun_out/verify_bench.log
cd /tmp && export TMPDIR=/tmp && cd $R && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/verify_prof -o run -- python bench.py --steps 10 --warmup 3 > gpurun_out/verify_prof.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/verify_prof.log; exit 1; }
echo ALL_OK
