set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R && python -m triton_client_amd._build
cd $R && timeout -k 10 500 python -m pytest tests/ -q -m gpu > gpurun_out/test_gpu_all.log 2>&1; echo "tests rc=$?"
cd $R && timeout -k 10 400 python tools/bench_conv.py > gpurun_out/bench_conv.log 2>&1; echo "conv rc=$?"
cd $R && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --only lidar > gpurun_out/bench_lid2.log 2>&1; echo "lid rc=$?"
