# fp32-input xb tiles for N <= 32 (88, 89) vs the v1 register-staging kernel (tile 0 auto) on the camera layers.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 500 python tools/bench_conv_x3.py 0,88,89 y > gpurun_out/xb_n32.jsonl 2> gpurun_out/xb_n32.err || { echo FAILED; tail -20 gpurun_out/xb_n32.err; exit 1; }
cut -c1-300 gpurun_out/xb_n32.jsonl
