# PMC of the halo-tiled conv (tile 90) vs the xb default (tile 70) on pp.b2.conv, pair storage.
set -o pipefail
R=$GRAFT_REPO_ROOT
cd $R
LAYER=pp.b2.conv TILE=90 PREC=fp32p bash tools/gpu_conv_pmc.sh && LAYER=pp.b2.conv TILE=70 PREC=fp32p bash tools/gpu_conv_pmc.sh
