#!/bin/bash
# Round-end measurement, part A (run on the GPU box from the repo root):
#   profiles/final_a.sh <tag>
# the default bench line (with the CPU baselines), a kernel trace of the
# default bench step, a kernel trace of C3 (100k random13), and the 8-rank
# one-GPU emulation of the sharded step (wide16 and skew) -> gpurun_out/<tag>_*
set -e -o pipefail
TAG=${1:?tag}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT"
timeout -k 10 400 python -u bench.py > "$OUT/${TAG}_bench.json" 2> "$OUT/${TAG}_bench.err"
timeout -k 10 300 python -u profiles/emulate_shards.py --world 8 --steps 3 --out "$OUT/${TAG}_shard_emulation.json" > "$OUT/${TAG}_emu.log" 2>&1
timeout -k 10 300 python -u profiles/emulate_shards.py --world 8 --steps 3 --kind skew --out "$OUT/${TAG}_shard_emulation_skew.json" > "$OUT/${TAG}_emu_skew.log" 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_trace" -o run -- \
    python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu --no-extras > "$OUT/${TAG}_trace.json" 2> "$OUT/${TAG}_trace.err"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_c3" -o run -- \
    python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu --no-extras --kind random13 --rows-per-gpu 100000 \
    > "$OUT/${TAG}_c3.json" 2> "$OUT/${TAG}_c3.err"
