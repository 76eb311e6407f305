#!/bin/bash
# Final-tree evidence after the vertex buffer placement (run from the repo root,
#   profiles/r06/r06ba_final.sh <tag>):
# profiles/collect.sh (trace + stats, FETCH/WRITE_SIZE passes, side kernels,
# store ceiling), C4 and C3 kernel traces, the C++ mirror, the 4- and 8-rank
# one-GPU emulation -> gpurun_out/prof_r06ba/, gpurun_out/${TAG}_*
set -e -o pipefail
TAG=${1:-r06ba}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 120 tests/cpp/test_graph_layout > "$OUT/${TAG}_cxx.log" 2>&1
bash profiles/collect.sh $TAG
cd "$ROOT"
timeout -k 10 300 python -u profiles/emulate_shards.py --world 8 --steps 3 --out "$OUT/${TAG}_emu_w8.json" > "$OUT/${TAG}_emu_w8.log" 2>&1
timeout -k 10 300 python -u profiles/emulate_shards.py --world 4 --steps 3 --out "$OUT/${TAG}_emu_w4.json" > "$OUT/${TAG}_emu_w4.log" 2>&1
cd /tmp && export TMPDIR=/tmp
BENCH="$ROOT/bench.py --steps 5 --no-cpu --no-extras"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_c4" -o run -- \
    python3 $BENCH --warmup 6 --kind linux --rows-per-gpu 1300000 > "$OUT/${TAG}_c4.json" 2> "$OUT/${TAG}_c4.err"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_c3" -o run -- \
    python3 $BENCH --warmup 2 --kind random13 --rows-per-gpu 100000 > "$OUT/${TAG}_c3.json" 2> "$OUT/${TAG}_c3.err"
