set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R && python -m triton_client_amd._build
cd $R && timeout -k 10 300 python bench.py --steps 30 --warmup 5 --only camera > gpurun_out/bench11_cam.log 2>&1; echo "cam rc=$?"
cd $R && timeout -k 10 300 python bench.py --steps 30 --warmup 5 --only lidar > gpurun_out/bench11_lid.log 2>&1; echo "lid rc=$?"
cd /tmp && export TMPDIR=/tmp && cd $R && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof11c -o run -- python bench.py --steps 10 --warmup 3 --only camera > gpurun_out/prof11c.log 2>&1; echo "profc rc=$?"
cd /tmp && export TMPDIR=/tmp && cd $R && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof11l -o run -- python bench.py --steps 10 --warmup 3 --only lidar > gpurun_out/prof11l.log 2>&1; echo "profl rc=$?"
