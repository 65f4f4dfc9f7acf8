#!/usr/bin/env bash
# Deploy served models into a (local or remote) model repository — the
# reference's deploy.sh:1-65 flow (export model, write config.pbtxt, copy into
# the server's repository over ssh), MI355X-native: no ONNX export, the server
# runs the in-tree HIP pipelines; the repository carries each model's KServe
# contract and, optionally, its state_dict (path or file/http(s)/s3 URI).
#
#   ./deploy.sh [-m MODELS] [-w MODEL=URI]... [-s MODEL=SHA256]... [-r user@host] [-d REMOTE_DIR] [OUT_DIR]
#
# No credentials are read or written here; s3:// weights are fetched by the
# server at load time with env-provided keys (utils/model_store.py) and
# checked against the -s sha256 (local files get theirs recorded automatically).
set -euo pipefail
MODELS="YOLOv5nCOCO,pointpillar_kitti"
REMOTE=""
REMOTE_DIR="/models"
WEIGHTS=()
while getopts "m:w:s:r:d:h" opt; do
  case "$opt" in
    m) MODELS="$OPTARG" ;;
    w) WEIGHTS+=(--weights "$OPTARG") ;;
    s) WEIGHTS+=(--weights-sha256 "$OPTARG") ;;
    r) REMOTE="$OPTARG" ;;
    d) REMOTE_DIR="$OPTARG" ;;
    *) sed -n '2,12p' "$0"; exit 0 ;;
  esac
done
shift $((OPTIND - 1))
OUT="${1:-./model_repository}"
cd "$(dirname "$0")"
python -m triton_client_amd.server --export-repository "$OUT" --models "$MODELS" "${WEIGHTS[@]}"
if [[ -n "$REMOTE" ]]; then
  ssh "$REMOTE" mkdir -p "$REMOTE_DIR"
  scp -r "$OUT"/. "$REMOTE:$REMOTE_DIR/"
  echo "deployed $MODELS to $REMOTE:$REMOTE_DIR"
else
  echo "model repository written to $OUT (serve: python -m triton_client_amd.server --model-repository $OUT)"
fi
