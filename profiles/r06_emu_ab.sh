#!/bin/bash
# sharded-step emulation (8 x 1M wide16) alternating two engine builds in one
# call: profiles/r06_emu_ab.sh <tag> <lib_a> <lib_b> [pairs] -> gpurun_out/<tag>_{a,b}<i>.json
set -e -o pipefail
TAG=${1:?tag}; A=${2:?lib a}; B=${3:?lib b}; PAIRS=${4:-2}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT"
for i in $(seq 1 "$PAIRS"); do
    for v in a b; do
        if [ "$v" = a ]; then L=$A; else L=$B; fi
        WGRAPH_LIB=$L timeout -k 10 300 python -u profiles/emulate_shards.py --world 8 --steps 3 \
            --out "$OUT/${TAG}_${v}${i}.json" > "$OUT/${TAG}_${v}${i}.log" 2>&1
    done
done
