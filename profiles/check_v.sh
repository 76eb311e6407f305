#!/bin/bash
# One validation + measurement pass of the tree (run on the GPU box from the
# repo root): profiles/check_v.sh <tag>
#   gpu_validate.sh (C++ mirror tests, GPU parity tests, wide16 kernel trace),
#   the lane stage on skew / linuxwide, and kernel traces of C3 (100k
#   random13) and linuxwide -> gpurun_out/<tag>_*
# Each step under its own time limit; the first failure ends the script.
set -e -o pipefail
TAG=${1:?tag}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
cd "$ROOT"
bash profiles/gpu_validate.sh "$TAG"
cd "$ROOT"
timeout -k 10 300 python -u profiles/lane_paths.py 3 skew,linuxwide > "$OUT/${TAG}_lanes.jsonl" 2> "$OUT/${TAG}_lanes.err"
timeout -k 10 300 python -u bench.py --no-cpu > "$OUT/${TAG}_bench.json" 2> "$OUT/${TAG}_bench.err"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_c3" -o run -- \
    python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu --no-extras --kind random13 --rows-per-gpu 100000 \
    > "$OUT/${TAG}_c3.json" 2> "$OUT/${TAG}_c3.err"
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_lw" -o run -- \
    python3 "$ROOT/bench.py" --steps 3 --warmup 1 --no-cpu --no-extras --kind linuxwide \
    > "$OUT/${TAG}_lw.json" 2> "$OUT/${TAG}_lw.err"
