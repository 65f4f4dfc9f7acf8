set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R && python -m triton_client_amd._build
cd $R && timeout -k 10 600 python -m pytest tests/ -q -m gpu > gpurun_out/test_gpu_all4.log 2>&1; echo "tests rc=$?"
cd $R && timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench6.log 2>&1; echo "bench rc=$?"
cd $R && timeout -k 10 300 python bench.py --steps 30 --warmup 5 --serial > gpurun_out/bench6_serial.log 2>&1; echo "serial rc=$?"
cd $R && timeout -k 10 300 python bench.py --steps 30 --warmup 5 --serial --no-prefetch > gpurun_out/bench6_plain.log 2>&1; echo "plain rc=$?"
cd /tmp && export TMPDIR=/tmp && cd $R && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof6 -o run -- python bench.py --steps 10 --warmup 3 > gpurun_out/prof6.log 2>&1; echo "prof rc=$?"
