set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R && python -m triton_client_amd._build
cd $R && timeout -k 10 500 python -m pytest tests/ -q -m gpu > gpurun_out/test_gpu_all2.log 2>&1; echo "tests rc=$?"
cd $R && timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench4.log 2>&1; echo "bench rc=$?"
cd $R && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --only camera > gpurun_out/bench4_cam.log 2>&1; echo "cam rc=$?"
cd $R && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --only lidar > gpurun_out/bench4_lid.log 2>&1; echo "lid rc=$?"
cd /tmp && export TMPDIR=/tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof3 -o bench -- python $R/bench.py --steps 10 --warmup 3 > $R/gpurun_out/prof3.log 2>&1
echo "done rc=$?"
