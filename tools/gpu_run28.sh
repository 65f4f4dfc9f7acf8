set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R && python -m triton_client_amd._build > gpurun_out/build28.log 2>&1
cd $R && timeout -k 10 600 python -m pytest tests/test_ops_gpu.py tests/test_fast_plans.py tests/test_pipelines_gpu.py tests/test_drivers_gpu.py -q -x -m gpu > gpurun_out/test28.log 2>&1
cd $R && timeout -k 10 600 python tools/bench_conv.py > gpurun_out/bench_conv_v6.jsonl 2>&1
cd $R && timeout -k 10 300 python bench.py --steps 40 --warmup 5 --only camera > gpurun_out/bench28_cam.log 2>&1
cd $R && timeout -k 10 300 python bench.py --steps 40 --warmup 5 > gpurun_out/bench28.log 2>&1
cd $R && timeout -k 10 300 python bench.py --steps 40 --warmup 5 > gpurun_out/bench28b.log 2>&1
cd /tmp && export TMPDIR=/tmp && cd $R && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof28c -o run -- python bench.py --steps 10 --warmup 3 --only camera > gpurun_out/prof28c.log 2>&1
