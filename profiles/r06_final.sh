#!/bin/bash
# Round-6 measurement set on one box, at the final code (run from the repo root):
#   profiles/r06_final.sh <tag>
# 1. the default bench line (CPU legs included), as the driver runs it;
# 2. rocprofv3 kernel trace + stats of the default step and of C4 (Linux-shaped 1.3M);
# 3. PMC passes of the emission (FETCH_SIZE / WRITE_SIZE, separate runs);
# 4. the 8-rank one-GPU emulation (lockstep segments + isolated per-rank replay), world 4 and 8.
# -> gpurun_out/<tag>_*
set -e -o pipefail
TAG=${1:?tag}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python -u bench.py > "$OUT/${TAG}_bench.json" 2> "$OUT/${TAG}_bench.err"
timeout -k 10 300 python -u profiles/emulate_shards.py --world 8 --steps 3 --out "$OUT/${TAG}_emu_w8.json" > "$OUT/${TAG}_emu_w8.log" 2>&1
timeout -k 10 300 python -u profiles/emulate_shards.py --world 4 --steps 3 --out "$OUT/${TAG}_emu_w4.json" > "$OUT/${TAG}_emu_w4.log" 2>&1
cd /tmp && export TMPDIR=/tmp
BENCH="$ROOT/bench.py --steps 5 --warmup 2 --no-cpu --no-extras"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_trace" -o run -- \
    python3 $BENCH > "$OUT/${TAG}_trace.json" 2> "$OUT/${TAG}_trace.err"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_c4" -o run -- \
    python3 $BENCH --warmup 6 --kind linux --rows-per-gpu 1300000 > "$OUT/${TAG}_c4.json" 2> "$OUT/${TAG}_c4.err"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_c3" -o run -- \
    python3 $BENCH --kind random13 --rows-per-gpu 100000 > "$OUT/${TAG}_c3.json" 2> "$OUT/${TAG}_c3.err"
timeout -s KILL 120 rocprofv3 --kernel-include-regex k_vtx_tile --pmc FETCH_SIZE --output-format csv -d "$OUT/${TAG}_fetch" -o run -- \
    python3 $BENCH > "$OUT/${TAG}_fetch.json" 2> "$OUT/${TAG}_fetch.err"
timeout -s KILL 120 rocprofv3 --kernel-include-regex k_vtx_tile --pmc WRITE_SIZE --output-format csv -d "$OUT/${TAG}_write" -o run -- \
    python3 $BENCH > "$OUT/${TAG}_write.json" 2> "$OUT/${TAG}_write.err"
