#!/bin/bash
# Profile collection for one round (run on the GPU box from the repo root):
#   profiles/collect.sh r01
# 1. rocprofv3 --kernel-trace --stats of the default bench command;
# 2. PMC passes for the dominant kernel (k_vtx_tile), one counter group per
#    run and kernel trace only (MI355X_MICROARCH.md §HBM: FETCH_SIZE and
#    WRITE_SIZE cannot share a pass; never combined with sys/runtime traces);
# 3. kernel statistics of the full bench (side measurements: glyph quads,
#    atlas, search, order) and the store-bandwidth ceiling microbenchmark;
# 4. profiles/summarize.py turns them into <tag>_kernels.md / <tag>_pmc.json /
#    <tag>_side_kernels.md / <tag>_store_ceiling.jsonl.
# Everything lands in gpurun_out/prof_<tag>/; the summaries are then copied
# into profiles/ by hand and committed.
set -e -o pipefail
TAG=${1:-r01}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/prof_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
BENCH="$ROOT/bench.py --steps 5 --warmup 2 --no-cpu --no-extras"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $BENCH > "$OUT/trace.json" 2> "$OUT/trace.err"
timeout -k 10 300 rocprofv3 --kernel-include-regex k_vtx_tile --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 $BENCH > "$OUT/fetch.json" 2> "$OUT/fetch.err"
timeout -k 10 300 rocprofv3 --kernel-include-regex k_vtx_tile --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 $BENCH > "$OUT/write.json" 2> "$OUT/write.err"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/side" -o run -- python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu > "$OUT/side.json" 2> "$OUT/side.err"
if [ -x "$ROOT/profiles/microbench/store_ceiling" ]; then
    timeout -k 10 120 "$ROOT/profiles/microbench/store_ceiling" > "$OUT/store_ceiling.jsonl" 2> "$OUT/store_ceiling.err"
    # the same timed with device-scope events, as bench.py times the emission
    STORE_EVENTS=device timeout -k 10 120 "$ROOT/profiles/microbench/store_ceiling" > "$OUT/store_ceiling_devev.jsonl" 2>> "$OUT/store_ceiling.err"
fi
if [ -x "$ROOT/profiles/microbench/store_sweep" ]; then
    timeout -k 10 200 "$ROOT/profiles/microbench/store_sweep" > "$OUT/store_sweep.jsonl" 2> "$OUT/store_sweep.err"
fi
python3 "$ROOT/profiles/summarize.py" "$OUT" "$TAG"
