set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R && python -m triton_client_amd._build
cd $R && timeout -k 10 400 python -m pytest tests/test_pipelines_gpu.py -q -m gpu > gpurun_out/test_pipe.log 2>&1; echo "tests rc=$?"
cd $R && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --only camera > gpurun_out/bench_cam.log 2>&1; echo "cam rc=$?"
cd $R && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --only lidar > gpurun_out/bench_lid.log 2>&1; echo "lid rc=$?"
cd /tmp && export TMPDIR=/tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof2 -o bench -- python $R/bench.py --steps 10 --warmup 3 > $R/gpurun_out/prof2.log 2>&1
echo "done rc=$?"
