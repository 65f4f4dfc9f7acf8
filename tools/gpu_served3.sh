set -o pipefail
cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out
timeout -k 10 300 python tools/served_bench.py --frames 256 --window 8 --client-procs 2 --wire shm > gpurun_out/served3_p2.log 2>&1; echo rc=$?
grep -v "amdgpu.ids" gpurun_out/served3_p2.log | head -80
