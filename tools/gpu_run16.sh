set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R && python -m triton_client_amd._build
cd $R && timeout -k 10 600 python -m pytest tests/test_yolov4.py tests/test_detectron.py -q -x > gpurun_out/test_y4det.log 2>&1; echo "tests rc=$?"
cd $R && timeout -k 10 400 python bench.py --steps 10 --warmup 3 --only camera --camera-model yolov4 > gpurun_out/bench_y4.log 2>&1; echo "y4 rc=$?"
