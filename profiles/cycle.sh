#!/bin/bash
# One GPU check of the tree (run on the GPU box from the repo root):
#   profiles/cycle.sh <tag> [pytest selection]
# the -m gpu tests, the default bench line (no CPU baseline) and one
# rocprofv3 kernel trace of a short bench -> gpurun_out/<tag>/
set -e -o pipefail
TAG=${1:?tag}
SEL=${2:-tests}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 600 python -u -m pytest $SEL -m gpu -x -v --timeout 300 --timeout-method thread > "$OUT/t.log" 2>&1
timeout -k 10 240 python bench.py --no-cpu > "$OUT/bench.json" 2> "$OUT/bench.err"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu --no-extras > "$OUT/trace.json" 2>&1
# C3 (100k random13, launch-bound) trace
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace_c3" -o run -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu --no-extras --kind random13 --rows-per-gpu 100000 > "$OUT/trace_c3.json" 2>&1
