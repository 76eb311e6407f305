#!/bin/bash
# quick GPU validation of a change (run from the repo root):
#   profiles/r06_check.sh <tag> [pytest files...]
# the named GPU tests, a short bench line (no CPU legs) and a kernel trace of
# the default step -> gpurun_out/<tag>_*
set -e -o pipefail
TAG=${1:?tag}; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT"
if [ $# -gt 0 ]; then
    timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread "$@" > "$OUT/${TAG}_tests.log" 2>&1
fi
timeout -k 10 300 python -u bench.py --no-cpu > "$OUT/${TAG}_bench.json" 2> "$OUT/${TAG}_bench.err"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_trace" -o run -- \
    python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu --no-extras > "$OUT/${TAG}_trace.json" 2> "$OUT/${TAG}_trace.err"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_c4" -o run -- \
    python3 "$ROOT/bench.py" --steps 5 --warmup 4 --no-cpu --no-extras --kind linux --rows-per-gpu 1300000 \
    > "$OUT/${TAG}_c4.json" 2> "$OUT/${TAG}_c4.err"
