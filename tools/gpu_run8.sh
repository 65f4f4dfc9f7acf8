set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R && python -m triton_client_amd._build
cd $R && timeout -k 10 300 python tools/debug_determinism.py > gpurun_out/det.log 2>&1; echo "det rc=$?"
cd $R && timeout -k 10 500 python -m pytest tests/ -q -m gpu > gpurun_out/test_gpu_all3.log 2>&1; echo "tests rc=$?"
cd $R && timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench5.log 2>&1; echo "bench rc=$?"
cd $R && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --only lidar > gpurun_out/bench5_lid.log 2>&1; echo "lid rc=$?"
