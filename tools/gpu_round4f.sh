# Round-4 GPU check, part 6: fused C3 tests / layer table / benches, neck tiling variants, and the
# bench.py multi-rank rehearsal (gloo, 2 and 4 ranks on the one card).
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4
mkdir -p $O
cd $R
fatal() { case $1 in 124|134|137|139) echo "FATAL rc=$1 in $2: stopping"; exit $1;; esac; }
bash tools/gpu_c3f.sh; rc=$?
fatal $rc c3f
echo "== hx3 16-line tiles"
timeout -k 10 400 python -u -m pytest tests/test_hx3_gpu.py -q -m gpu --timeout 300 --timeout-method thread -k "117 or 118" > $O/pytest_hx3_16.log 2>&1; rc=$?
tail -2 $O/pytest_hx3_16.log
fatal $rc hx3_16
timeout -k 10 300 python -u tools/bench_conv_x3.py 0,115,116,117,118 pp.b1.conv --pair > $O/hx3_16_tiles.jsonl 2>&1; rc=$?
grep layer $O/hx3_16_tiles.jsonl
fatal $rc hx3_16_tiles
echo "== neck variants"
timeout -k 10 300 python -u tools/bench_neck.py 32 1,2,3,4,5 > $O/neck_variants.jsonl 2>&1; rc=$?
cat $O/neck_variants.jsonl | tail -8
fatal $rc neck
echo "== bench.py rehearsal"
timeout -k 10 900 bash tools/gpu_dp_rehearsal.sh; rc=$?
fatal $rc dp_rehearsal
echo "== served (shm / raw, one and two server processes)"
NOTEST=1 SPROCS=1 TAG=_r4f timeout -k 10 400 bash tools/gpu_served3.sh; rc=$?
fatal $rc served1
NOTEST=1 SPROCS=2 TAG=_r4f timeout -k 10 400 bash tools/gpu_served3.sh; rc=$?
fatal $rc served2
