set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R && python -m triton_client_amd._build > gpurun_out/build21.log 2>&1
cd $R && timeout -k 10 600 python -m pytest tests/test_neck.py tests/test_fast_plans.py tests/test_pipelines_gpu.py -q -x -m gpu > gpurun_out/test21.log 2>&1
cd $R && timeout -k 10 300 python bench.py --steps 30 --warmup 5 --only lidar > gpurun_out/bench21_lid.log 2>&1
cd $R && timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench21.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $R && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof21l -o run -- python bench.py --steps 10 --warmup 3 --only lidar > gpurun_out/prof21l.log 2>&1
