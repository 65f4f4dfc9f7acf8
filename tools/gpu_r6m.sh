# Round 6: PillarVFE two pillars per wave iteration (TCA_VFE_LIN2=1, variant 2): the VFE tests (numerics
# vs fp32 and vs the one-pillar kernel), standalone VFE times of the three variants
# (tools/bench_vfe.py), then same-box LiDAR-only and headline A/Bs of the switch.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/r6/vfe2
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -k "pillar_vfe" -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/r6/vfe2/tests.log 2>&1 || { echo TESTS_FAILED; grep -E "FAILED|Error|assert" gpurun_out/r6/vfe2/tests.log | tail -20; exit 1; }
tail -1 gpurun_out/r6/vfe2/tests.log
for v in lin lin2 mfma lin lin2; do
  timeout -k 10 200 python tools/bench_vfe.py --variant $v --reps 30 >> gpurun_out/r6/vfe2/bench_vfe.jsonl 2> gpurun_out/r6/vfe2/bench_vfe_$v.err || { echo VFE_BENCH_FAILED $v; tail -20 gpurun_out/r6/vfe2/bench_vfe_$v.err; exit 1; }
  tail -1 gpurun_out/r6/vfe2/bench_vfe.jsonl
done
VAR=TCA_VFE_LIN2 A= B=1 RUNS=2 TAG=vfe2_lidar EXTRA="--only lidar" bash tools/gpu_env_ab.sh || exit 1
VAR=TCA_VFE_LIN2 A= B=1 RUNS=3 TAG=vfe2_head bash tools/gpu_env_ab.sh || exit 1
