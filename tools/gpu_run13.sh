set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R && python -m triton_client_amd._build
cd $R && timeout -k 10 600 python tools/reference_equivalent.py --frames 5 --device cuda --json-out gpurun_out/refeq.json > gpurun_out/refeq.log 2>&1; echo "refeq rc=$?"
cd $R && timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench9.log 2>&1; echo "bench rc=$?"
cd /tmp && export TMPDIR=/tmp && cd $R && timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof9 -o run -- python bench.py --steps 10 --warmup 3 > gpurun_out/prof9.log 2>&1; echo "prof rc=$?"
