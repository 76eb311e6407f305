#!/bin/bash
# One GPU validation pass (run on the box from the repo root): the C++
# mirror's tests, the layout / lanes / frames / shard GPU tests, then a kernel
# trace of the default bench command.  Each step under its own time limit;
# the first failure ends the script.
set -e -o pipefail
TAG=${1:-val}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out
mkdir -p "$OUT"
timeout -k 10 120 "$ROOT/tests/cpp/test_graph_layout" > "$OUT/${TAG}_cxx.log" 2>&1
timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_lane_pins.py tests/test_gpu_spec.py \
    tests/test_gpu_lanes_wide.py tests/test_gpu_frames.py tests/test_gpu_shard.py -x -q --timeout 300 \
    --timeout-method thread > "$OUT/${TAG}_tests.log" 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${TAG}_prof" -o run -- \
    python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu --no-extras > "$OUT/${TAG}_prof.json" 2> "$OUT/${TAG}_prof.err"
