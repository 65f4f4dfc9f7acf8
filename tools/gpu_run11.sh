set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R && python -m triton_client_amd._build
cd $R && timeout -k 10 300 python -m pytest tests/test_ops_gpu.py -q -x -k conv > gpurun_out/test_conv_v3.log 2>&1; echo "conv tests rc=$?"
cd $R && timeout -k 10 400 python tools/bench_conv.py > gpurun_out/bench_conv_v3.log 2>&1; echo "bench_conv rc=$?"
