# PMC passes for the pair-storage conv kernels (tools/gpu_conv_pmc.sh per layer / tile).
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
LAYER=pp.b2.conv TILE=20 PREC=fp32p bash tools/gpu_conv_pmc.sh && LAYER=pp.b1.conv TILE=26 PREC=fp32p bash tools/gpu_conv_pmc.sh && LAYER=pp.b1.conv TILE=41 PREC=fp32 bash tools/gpu_conv_pmc.sh
