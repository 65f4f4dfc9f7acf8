set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/r5
timeout -k 10 300 python -u -m pytest tests/test_fp32_mode_gpu.py -x -q -m gpu -k "neck" --timeout 200 --timeout-method thread > gpurun_out/r5/neck4_tests.log 2>&1 || { echo TESTS_FAILED; tail -20 gpurun_out/r5/neck4_tests.log; exit 1; }
tail -1 gpurun_out/r5/neck4_tests.log
timeout -k 10 200 python tools/bench_neck.py 32 0,1,2 > gpurun_out/r5/neck4_bench.log 2>&1 || { echo NECK_FAILED; tail -20 gpurun_out/r5/neck4_bench.log; exit 1; }
tail -1 gpurun_out/r5/neck4_bench.log
TAG=neck4 VAR=TCA_NECK_VARIANT A=0 B=2 RUNS=3 bash tools/gpu_env_ab.sh
