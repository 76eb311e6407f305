#!/bin/bash
# rocprofv3 kernel statistics of the full bench (side measurements included):
#   bash profiles/prof_stats.sh <outdir-under-gpurun_out>
set -e -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/${1:-stats}
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu > "$OUT/bench.json" 2> "$OUT/bench.err"
