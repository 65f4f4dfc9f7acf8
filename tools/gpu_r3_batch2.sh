# Round 3 batch 2: hx3 on by default -> PMC of the hx3 tiles, the LiDAR / camera step profiles
# and the headline bench, then the failing batch-1 tests again.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
cd $R
timeout -k 10 300 python -u -m pytest tests/test_hx3_gpu.py "tests/test_detectron.py::test_served_test_model_fp32_matches_local_engine" "tests/test_fp32_mode_gpu.py::test_pipeline_fp32_detection_parity_headline_shape" -v -m gpu --timeout 200 --timeout-method thread > gpurun_out/r3b2_tests.log 2>&1; echo "tests rc=$?"
grep -E "passed|failed" gpurun_out/r3b2_tests.log | tail -2
TAG=r3_hx3 bash tools/gpu_step_profile.sh || exit 1
for lt in "pp.b2.conv 110" "pp.b1.conv 114" "pp.b3.conv 110"; do
  set -- $lt
  LAYER=$1 TILE=$2 PREC=fp32p bash tools/gpu_conv_pmc.sh > gpurun_out/pmc_$1_$2.log 2>&1 || { echo PMC_FAILED $lt; tail -5 gpurun_out/pmc_$1_$2.log; exit 1; }
  python tools/pmc_summary.py conv_hx3 gpurun_out/pmc/$1_$2_fp32p_p*.csv > gpurun_out/pmc_hx3_$1.md || exit 1
  grep -E "MFMA busy|wave time|VALU per|bank" gpurun_out/pmc_hx3_$1.md
done
