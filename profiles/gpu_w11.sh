#!/bin/bash
# r05: step timelines (kernel trace) of C3 (100k random13) and the wide16 headline, for the gap analysis
set -e -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/w11
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/c3" -o run -- python3 "$ROOT/bench.py" --steps 8 --warmup 3 --no-cpu --no-extras --no-events --kind random13 --rows-per-gpu 100000 > "$OUT/c3.json" 2> "$OUT/c3.err"
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/w16" -o run -- python3 "$ROOT/bench.py" --steps 8 --warmup 3 --no-cpu --no-extras --no-events > "$OUT/w16.json" 2> "$OUT/w16.err"
cd "$ROOT"
for k in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 50 --no-cpu --no-extras --kind random13 --rows-per-gpu 100000 > $OUT/c3_$k.json 2> $OUT/c3_$k.err
done
