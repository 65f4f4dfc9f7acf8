# LiDAR software pipeline A/B (MODES: --lidar-pipeline values, e.g. "3 2 1 0"; LMODE: the mode of the
# LiDAR-only, 2-rank gloo rehearsal and trace runs): GPU pipeline tests, headline A/B x2.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_pipelines_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lpipe2_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/lpipe2_tests.log; exit 1; }
tail -1 gpurun_out/lpipe2_tests.log
for k in 1 2; do
for p in ${MODES:-3 0}; do
  timeout -k 10 300 python bench.py --steps 50 --warmup 10 --lidar-pipeline $p > gpurun_out/lpipe2_$p.log 2>&1 || { echo BENCH_FAILED $p; tail -30 gpurun_out/lpipe2_$p.log; exit 1; }
  echo "pipeline=$p $(tail -1 gpurun_out/lpipe2_$p.log | cut -c100-200) $(grep -o '"lidar_pipelined": "[a-z]*"' gpurun_out/lpipe2_$p.log) 3d=$(grep -o '"avg_3d_dets_per_frame": [0-9.]*' gpurun_out/lpipe2_$p.log) 2d=$(grep -o '"avg_2d_dets_per_frame": [0-9.]*' gpurun_out/lpipe2_$p.log)"
done
done
timeout -k 10 300 python bench.py --only lidar --steps 30 --warmup 5 --lidar-pipeline ${LMODE:-3} > gpurun_out/lpipe2_lid.log 2>&1 || { echo BENCH_FAILED lid; tail -30 gpurun_out/lpipe2_lid.log; exit 1; }
echo "lidar only mode $LMODE $(tail -1 gpurun_out/lpipe2_lid.log | cut -c100-200)"
TCA_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29614 bench.py --gpus 2 --steps 5 --warmup 2 --lidar-pipeline ${LMODE:-3} > gpurun_out/lpipe2_dp2.log 2>&1 || { echo DP_FAILED; tail -30 gpurun_out/lpipe2_dp2.log; exit 1; }
echo "dp2 $(grep '^{' gpurun_out/lpipe2_dp2.log | cut -c100-200) 3d=$(grep -o '"avg_3d_dets_per_frame": [0-9.]*' gpurun_out/lpipe2_dp2.log)"
cd /tmp && export TMPDIR=/tmp && cd $R
rm -rf /tmp/lp2_full
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/lp2_full -o run -- python bench.py --steps 8 --warmup 3 --lidar-pipeline ${LMODE:-3} > gpurun_out/lpipe2_full.log 2>&1 || { echo PROF_FAILED; tail -20 gpurun_out/lpipe2_full.log; exit 1; }
f=$(find /tmp/lp2_full -name "*kernel_trace.csv" | head -1)
python tools/step_stats.py $f --marker yolo_stem --steps 6 --sequence > gpurun_out/lpipe2_full_steps.txt || exit 1
head -3 gpurun_out/lpipe2_full_steps.txt
