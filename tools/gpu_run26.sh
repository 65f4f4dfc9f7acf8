set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R && python -m triton_client_amd._build > gpurun_out/build26.log 2>&1
cd $R && timeout -k 10 300 python tools/probe_vox.py > gpurun_out/probe_vox3.log 2>&1
cd $R && timeout -k 10 900 python -m pytest tests/ -q -x -m gpu > gpurun_out/test26.log 2>&1
cd $R && timeout -k 10 300 python bench.py --steps 30 --warmup 5 --only lidar > gpurun_out/bench26_lid.log 2>&1
cd $R && timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench26.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $R && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof26l -o run -- python bench.py --steps 10 --warmup 3 --only lidar > gpurun_out/prof26l.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $R && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof26c -o run -- python bench.py --steps 10 --warmup 3 --only camera > gpurun_out/prof26c.log 2>&1
