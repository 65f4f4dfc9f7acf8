set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R && python -m triton_client_amd._build > gpurun_out/build19.log 2>&1
cd $R && timeout -k 10 600 python -m pytest tests/test_ops_gpu.py -q -x -k "glds_tiles" > gpurun_out/test19.log 2>&1
cd $R && timeout -k 10 600 python tools/bench_conv.py > gpurun_out/bench_conv_v5.jsonl 2>&1
