#!/bin/bash
# r05: the sweep at two waves per 64-row chunk (WG_SWEEP_SPLIT=1) — parity with it, then A/B
set -e -o pipefail
mkdir -p gpurun_out/w16
WG_SWEEP_SPLIT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_frames.py tests/test_gpu_lanes_wide.py -x -q --timeout 300 --timeout-method thread > gpurun_out/w16/tests.log 2>&1
for k in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 20 --no-cpu --no-extras > gpurun_out/w16/one_$k.json 2> gpurun_out/w16/one_$k.err
  WG_SWEEP_SPLIT=1 timeout -k 10 200 python -u bench.py --steps 20 --no-cpu --no-extras > gpurun_out/w16/two_$k.json 2> gpurun_out/w16/two_$k.err
done
