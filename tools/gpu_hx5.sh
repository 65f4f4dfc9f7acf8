# hx 4x2-wave variant (tile 102): halo tests for it, then the b2 / b3 sweep vs 94.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_pair_storage_gpu.py -x -v -m gpu -k "halo_tiles_vs_fp64 and 102" --timeout 120 --timeout-method thread > gpurun_out/hx5_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/hx5_tests.log; exit 1; }
tail -1 gpurun_out/hx5_tests.log
timeout -k 10 300 python tools/bench_conv_x3.py 0,94,102 pp.b2.conv,pp.b3.conv --pair > gpurun_out/hx5_tiles.jsonl 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/hx5_tiles.jsonl; exit 1; }
cut -c1-300 gpurun_out/hx5_tiles.jsonl
