set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R && python -m triton_client_amd._build > gpurun_out/build27.log 2>&1
cd $R && timeout -k 10 600 python -m pytest tests/test_ops_gpu.py tests/test_pipelines_gpu.py tests/test_centerpoint.py -q -x -m gpu > gpurun_out/test27.log 2>&1
cd $R && timeout -k 10 300 python bench.py --steps 40 --warmup 5 --only lidar > gpurun_out/bench27_lid.log 2>&1
cd $R && timeout -k 10 300 python bench.py --steps 40 --warmup 5 > gpurun_out/bench27.log 2>&1
cd $R && timeout -k 10 300 python bench.py --steps 40 --warmup 5 > gpurun_out/bench27b.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $R && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof27l -o run -- python bench.py --steps 10 --warmup 3 --only lidar > gpurun_out/prof27l.log 2>&1
