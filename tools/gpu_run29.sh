set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R && python -m triton_client_amd._build > gpurun_out/build29.log 2>&1
for i in 1 2 3; do
cd $R && timeout -k 10 300 python bench.py --steps 50 --warmup 5 --graph-mode split > gpurun_out/bench29_split$i.log 2>&1 || exit 1
cd $R && timeout -k 10 300 python bench.py --steps 50 --warmup 5 --graph-mode fork > gpurun_out/bench29_fork$i.log 2>&1 || exit 1
done
