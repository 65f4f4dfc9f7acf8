set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R && python -m triton_client_amd._build
cd $R && timeout -k 10 500 python -m pytest tests/test_detectron.py -q -x > gpurun_out/test_det.log 2>&1; echo "det tests rc=$?"
cd $R && timeout -k 10 400 python bench.py --steps 10 --warmup 3 --only camera --camera-model retinanet > gpurun_out/bench_retina.log 2>&1; echo "retina rc=$?"
cd $R && timeout -k 10 400 python bench.py --steps 10 --warmup 3 --only camera --camera-model fcos > gpurun_out/bench_fcos.log 2>&1; echo "fcos rc=$?"
