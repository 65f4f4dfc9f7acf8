set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R && python -m triton_client_amd._build
cd $R && timeout -k 10 900 python -m pytest tests/ -q -m gpu > gpurun_out/test_gpu_all6.log 2>&1; echo "tests rc=$?"
cd $R && timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench10.log 2>&1; echo "bench rc=$?"
