#!/bin/bash
# Validation + the lane stage on linuxwide / skew: profiles/check_z.sh <tag>  (GPU box, repo root)
set -e -o pipefail
TAG=${1:?tag}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
bash profiles/gpu_validate.sh "$TAG"
cd "$ROOT"
timeout -k 10 300 python -u profiles/lane_paths.py 3 linuxwide,skew > "$ROOT/gpurun_out/${TAG}_lanes.jsonl" 2> "$ROOT/gpurun_out/${TAG}_lanes.err"
