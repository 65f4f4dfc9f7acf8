# Round 6: private-memory fixes -- the fused YOLOv5 stem kept its hi / lo pixel halves and the
# RGB swap in scratch memory (80 B per lane per pixel), and the pair-input F(2,3) kernels called
# their transform as a function -- plus the two-pillar VFE.  Tests, then a same-box A/B of the
# build against the committed one (LiDAR-only + headline, 3 rounds, both LiDAR step tables), and
# camera-only runs of both.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/r6/fix
timeout -k 10 500 python -u -m pytest tests/test_stem_fused_gpu.py tests/test_wino_gpu.py tests/test_ops_gpu.py -x -q -m gpu -k "stem or wino or prep or preprocess or pillar_vfe or image" --timeout 200 --timeout-method thread > gpurun_out/r6/fix/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/r6/fix/tests.log | tail -20; tail -5 gpurun_out/r6/fix/tests.log; exit 1; }
tail -1 gpurun_out/r6/fix/tests.log
TAG=fix RUNS=3 STATS=1 bash tools/gpu_kernels_ab.sh || exit 1
BASE=$R/triton_client_amd/_lib/ab/libtca_kernels_base.so
for k in 1 2; do
  for L in new base; do
    if [ $L = base ]; then export TCA_KERNELS_LIB=$BASE; else unset TCA_KERNELS_LIB; fi
    timeout -k 10 300 python bench.py --only camera --steps 30 --warmup 5 > gpurun_out/r6/fix/cam_${L}_$k.log 2>&1 || { echo CAM_FAILED; tail -20 gpurun_out/r6/fix/cam_${L}_$k.log; exit 1; }
    echo "camera $L $k: $(tail -1 gpurun_out/r6/fix/cam_${L}_$k.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  done
done
unset TCA_KERNELS_LIB
