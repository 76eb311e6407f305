#!/bin/bash
# Validation + the 8-rank skew emulation: profiles/check_y.sh <tag>  (GPU box, repo root)
set -e -o pipefail
TAG=${1:?tag}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
bash profiles/gpu_validate.sh "$TAG"
cd "$ROOT"
timeout -k 10 300 python -u profiles/emulate_shards.py --world 8 --steps 2 --kind skew --out "$ROOT/gpurun_out/${TAG}_shard_emulation_skew.json" > "$ROOT/gpurun_out/${TAG}_emu_skew.log" 2>&1
