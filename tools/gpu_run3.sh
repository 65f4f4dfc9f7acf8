set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R && python -m triton_client_amd._build
cd $R && timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/bench2.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof -o bench -- python $R/bench.py --steps 10 --warmup 3 > $R/gpurun_out/prof.log 2>&1
echo "done rc=$?"
