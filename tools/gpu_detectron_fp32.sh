# Detectron2 RetinaNet / FCOS at fp32: GPU tests, then the camera-only bench at fp32 and bf16 (batch 16).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 600 python -u -m pytest tests/test_detectron.py -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/det_tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error" gpurun_out/det_tests.log | tail -20; tail -40 gpurun_out/det_tests.log; exit 1; }
tail -1 gpurun_out/det_tests.log
for arch in retinanet fcos; do
  for p in fp32 bf16; do
    timeout -k 10 300 python bench.py --only camera --camera-model $arch --batch 16 --steps 20 --warmup 5 --precision $p > gpurun_out/det_${arch}_$p.log 2>&1 || { echo BENCH_FAILED $arch $p; tail -20 gpurun_out/det_${arch}_$p.log; exit 1; }
    tail -1 gpurun_out/det_${arch}_$p.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$arch', d['dtype'], d['value'], d['ms_per_step'])"
  done
done
