set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R && python -m triton_client_amd._build
cd $R && timeout -k 10 400 python -m pytest tests/test_pipelines_gpu.py tests/test_ops_gpu.py -q -m gpu > gpurun_out/test_gpu.log 2>&1; echo "tests rc=$?"
cd $R && timeout -k 10 300 python tools/debug_lidar_bench.py > gpurun_out/dbg3.log 2>&1; echo "dbg rc=$?"
cd $R && timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench3.log 2>&1; echo "bench rc=$?"
