# hx after the conflict-free halo swizzle: correctness, tile sweep, PMC of tile 90.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
bash tools/gpu_hx.sh && LAYER=pp.b2.conv TILE=90 PREC=fp32p bash tools/gpu_conv_pmc.sh
