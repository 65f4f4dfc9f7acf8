set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R && python -m triton_client_amd._build
cd $R && timeout -k 10 400 python -m pytest tests/test_centerpoint.py tests/test_drivers_gpu.py -q -x > gpurun_out/test_cp.log 2>&1; echo "cp tests rc=$?"
cd $R && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --only lidar --lidar-model centerpoint > gpurun_out/bench_cp_lid.log 2>&1; echo "cp lid rc=$?"
cd $R && timeout -k 10 300 python bench.py --steps 20 --warmup 5 --lidar-model centerpoint > gpurun_out/bench_cp.log 2>&1; echo "cp both rc=$?"
