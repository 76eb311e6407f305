#!/bin/bash
# Final-tree evidence after the vertex buffer placement (run from the repo root):
# profiles/collect.sh (trace + stats, FETCH/WRITE_SIZE passes, side kernels,
# store ceiling), C4 and C3 kernel traces, the C++ mirror, the 4- and 8-rank
# one-GPU emulation -> gpurun_out/prof_r06ba/, gpurun_out/r06ba_*
set -e -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 120 tests/cpp/test_graph_layout > "$OUT/r06ba_cxx.log" 2>&1
bash profiles/collect.sh r06ba
cd "$ROOT"
timeout -k 10 300 python -u profiles/emulate_shards.py --world 8 --steps 3 --out "$OUT/r06ba_emu_w8.json" > "$OUT/r06ba_emu_w8.log" 2>&1
timeout -k 10 300 python -u profiles/emulate_shards.py --world 4 --steps 3 --out "$OUT/r06ba_emu_w4.json" > "$OUT/r06ba_emu_w4.log" 2>&1
cd /tmp && export TMPDIR=/tmp
BENCH="$ROOT/bench.py --steps 5 --no-cpu --no-extras"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/r06ba_c4" -o run -- \
    python3 $BENCH --warmup 6 --kind linux --rows-per-gpu 1300000 > "$OUT/r06ba_c4.json" 2> "$OUT/r06ba_c4.err"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/r06ba_c3" -o run -- \
    python3 $BENCH --warmup 2 --kind random13 --rows-per-gpu 100000 > "$OUT/r06ba_c3.json" 2> "$OUT/r06ba_c3.err"
