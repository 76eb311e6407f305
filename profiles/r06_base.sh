#!/bin/bash
# Round-6 starting point on one box (run from the repo root):
#   profiles/r06_base.sh <tag>
# default bench line, 8-rank one-GPU emulation (wide16), and kernel traces of
# the default step and of C4 (Linux-shaped 1.3M rows) -> gpurun_out/<tag>_*
set -e -o pipefail
TAG=${1:?tag}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python -u bench.py > "$OUT/${TAG}_bench.json" 2> "$OUT/${TAG}_bench.err"
timeout -k 10 300 python -u profiles/emulate_shards.py --world 8 --steps 3 --out "$OUT/${TAG}_shard_emulation.json" > "$OUT/${TAG}_emu.log" 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_trace" -o run -- \
    python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu --no-extras > "$OUT/${TAG}_trace.json" 2> "$OUT/${TAG}_trace.err"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_c4" -o run -- \
    python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu --no-extras --kind linux --rows-per-gpu 1300000 \
    > "$OUT/${TAG}_c4.json" 2> "$OUT/${TAG}_c4.err"
