# A/B: the persistent neck on all CUs vs a fraction of them (the rest left to the next batch's front).
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r4
cd $R
for rep in 1 2; do
  for f in 1.0 0.75 0.5; do
    for only in both lidar; do
      timeout -k 10 300 python -c "import sys, runpy; import triton_client_amd.ops.neck as n; n.NECK_CU_FRACTION = $f; sys.argv = ['bench.py', '--only', '$only', '--steps', '30', '--warmup', '10']; runpy.run_path('bench.py', run_name='__main__')" > gpurun_out/r4/ncu_${only}_${f}_$rep.log 2>&1 || { echo BENCH_FAILED; tail -20 gpurun_out/r4/ncu_${only}_${f}_$rep.log; exit 1; }
      echo "$rep $f $only $(tail -1 gpurun_out/r4/ncu_${only}_${f}_$rep.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
    done
  done
done
