set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R && python -m triton_client_amd._build > gpurun_out/build23.log 2>&1
cd $R && timeout -k 10 300 python tools/probe_nms.py > gpurun_out/probe_nms3.log 2>&1
cd $R && timeout -k 10 600 python -m pytest tests/test_ops_gpu.py tests/test_pipelines_gpu.py -q -x -m gpu > gpurun_out/test23.log 2>&1
cd $R && timeout -k 10 300 python bench.py --steps 30 --warmup 5 --only lidar > gpurun_out/bench23_lid.log 2>&1
cd $R && timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench23.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $R && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof23l -o run -- python bench.py --steps 10 --warmup 3 --only lidar > gpurun_out/prof23l.log 2>&1
