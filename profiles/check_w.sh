#!/bin/bash
# Validation (C++ mirror, GPU parity tests, wide16 trace) + a plain bench line:
#   profiles/check_w.sh <tag>   (GPU box, repo root)
set -e -o pipefail
TAG=${1:?tag}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
bash profiles/gpu_validate.sh "$TAG"
cd "$ROOT"
timeout -k 10 120 python -u bench.py --no-cpu --no-extras --steps 20 > "$ROOT/gpurun_out/${TAG}_bench.json" 2> "$ROOT/gpurun_out/${TAG}_bench.err"
timeout -k 10 120 python -u bench.py --no-cpu --no-extras --steps 20 > "$ROOT/gpurun_out/${TAG}_bench2.json" 2> "$ROOT/gpurun_out/${TAG}_bench2.err"
