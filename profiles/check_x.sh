#!/bin/bash
# Validation (C++ mirror, GPU parity tests, wide16 trace) + the bench line with
# the baseline configs (no CPU legs): profiles/check_x.sh <tag>  (GPU box, repo root)
set -e -o pipefail
TAG=${1:?tag}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
bash profiles/gpu_validate.sh "$TAG"
cd "$ROOT"
timeout -k 10 400 python -u bench.py --no-cpu > "$ROOT/gpurun_out/${TAG}_bench.json" 2> "$ROOT/gpurun_out/${TAG}_bench.err"
