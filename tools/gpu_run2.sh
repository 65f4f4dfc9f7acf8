set -o pipefail
mkdir -p gpurun_out
python -m triton_client_amd._build
timeout -k 10 300 python -m pytest tests/test_ops_gpu.py -q -m gpu > gpurun_out/test_ops_gpu.log 2>&1; echo "tests rc=$?"
timeout -k 10 300 python __graft_entry__.py --smoke > gpurun_out/smoke.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench1.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-graph --only lidar > gpurun_out/bench_lidar_eager.log 2>&1
echo "done rc=$?"
