#!/bin/bash
# Round-end measurement, part B (run on the GPU box from the repo root):
#   profiles/final_b.sh <tag>
# PMC passes, one counter group per run with kernel trace only
# (MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE in separate passes,
# never beside sys/runtime traces): the emission kernel (profiles/collect.sh)
# and the step's other kernels (profiles/pmc_step.sh).
set -e -o pipefail
TAG=${1:?tag}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
bash profiles/pmc_step.sh "$TAG"
cd "$ROOT"
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH="$ROOT/bench.py --steps 5 --warmup 2 --no-cpu --no-extras"
timeout -s KILL 120 rocprofv3 --kernel-include-regex k_vtx_tile --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 $BENCH > "$OUT/fetch.json" 2> "$OUT/fetch.err"
timeout -s KILL 120 rocprofv3 --kernel-include-regex k_vtx_tile --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 $BENCH > "$OUT/write.json" 2> "$OUT/write.err"
