#!/bin/bash
# Search kernel A/B of two engine builds, alternating processes (run from the repo root):
#   profiles/r06_match_ab.sh <tag> <lib_a> <lib_b> [pairs]  -> gpurun_out/<tag>_{a,b}<i>.jsonl
set -e -o pipefail
TAG=${1:?tag}; A=${2:?lib a}; B=${3:?lib b}; PAIRS=${4:-3}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT"
for i in $(seq 1 "$PAIRS"); do
    for v in a b; do
        if [ "$v" = a ]; then L=$A; else L=$B; fi
        WGRAPH_LIB=$L timeout -k 10 120 python -u profiles/match_probe.py > "$OUT/${TAG}_${v}${i}.jsonl" 2> "$OUT/${TAG}_${v}${i}.err"
    done
done
