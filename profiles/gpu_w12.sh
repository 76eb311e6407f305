#!/bin/bash
# r05: C3 step with the HIP API trace beside the kernel trace (what the host does in the lane stage's gap)
set -e -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/w12
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --hip-trace --output-format csv -d "$OUT/c3api" -o run -- python3 "$ROOT/bench.py" --steps 6 --warmup 3 --no-cpu --no-extras --no-events --kind random13 --rows-per-gpu 100000 > "$OUT/c3api.json" 2> "$OUT/c3api.err"
