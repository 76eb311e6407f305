#!/bin/bash
# r05: the sweep's output staged in LDS — geometry parity, then A/B (WG_SWEEP_NOSTAGE=1 = per-row stores)
set -e -o pipefail
mkdir -p gpurun_out/w13
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_frames.py tests/test_gpu_lanes_wide.py -x -q --timeout 300 --timeout-method thread > gpurun_out/w13/tests.log 2>&1
for k in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 20 --no-cpu --no-extras > gpurun_out/w13/stage_$k.json 2> gpurun_out/w13/stage_$k.err
  WG_SWEEP_NOSTAGE=1 timeout -k 10 200 python -u bench.py --steps 20 --no-cpu --no-extras > gpurun_out/w13/nostage_$k.json 2> gpurun_out/w13/nostage_$k.err
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/gpurun_out/w13/tr" -o run -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu --no-extras > "$GRAFT_REPO_ROOT/gpurun_out/w13/tr.json" 2>&1
