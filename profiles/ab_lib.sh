#!/bin/bash
# A/B of two engine builds in one call, alternating (run from the repo root):
#   profiles/ab_lib.sh <tag> <lib_a> <lib_b> [pairs]
# per pair and library: the default bench step (wide16 1M), C4 (Linux-shaped
# 1.3M) and C3 (random13 100k) [and skew 1M with AB_SKEW=1], 30 timed steps each, no CPU legs; then a
# kernel trace of the default step with lib_b -> gpurun_out/<tag>_*
set -e -o pipefail
TAG=${1:?tag}; A=${2:?lib a}; B=${3:?lib b}; PAIRS=${4:-3}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT"
for i in $(seq 1 "$PAIRS"); do
    for v in a b; do
        if [ "$v" = a ]; then L=$A; else L=$B; fi
        WGRAPH_LIB=$L timeout -k 10 120 python -u bench.py --no-cpu --no-extras --steps 30 \
            > "$OUT/${TAG}_${v}${i}_wide.json" 2> "$OUT/${TAG}_${v}${i}_wide.err"
        WGRAPH_LIB=$L timeout -k 10 120 python -u bench.py --no-cpu --no-extras --steps 30 --warmup 4 --kind linux \
            --rows-per-gpu 1300000 > "$OUT/${TAG}_${v}${i}_c4.json" 2> "$OUT/${TAG}_${v}${i}_c4.err"
        WGRAPH_LIB=$L timeout -k 10 120 python -u bench.py --no-cpu --no-extras --steps 30 --kind random13 \
            --rows-per-gpu 100000 > "$OUT/${TAG}_${v}${i}_c3.json" 2> "$OUT/${TAG}_${v}${i}_c3.err"
        if [ -n "$AB_SKEW" ]; then
            WGRAPH_LIB=$L timeout -k 10 120 python -u bench.py --no-cpu --no-extras --steps 30 --warmup 6 --kind skew \
                > "$OUT/${TAG}_${v}${i}_skew.json" 2> "$OUT/${TAG}_${v}${i}_skew.err"
        fi
    done
done
cd /tmp && export TMPDIR=/tmp
WGRAPH_LIB=$ROOT/$B timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_trace" -o run -- \
    python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu --no-extras > "$OUT/${TAG}_trace.json" 2> "$OUT/${TAG}_trace.err"
