#!/bin/bash
# r05 validation + A/B (run on the GPU box from the repo root)
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gpu_replay_forms.py tests/test_gpu_lanes_wide.py tests/test_lane_pins.py tests/test_gpu_spec.py tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread > gpurun_out/w3_tests.log 2>&1
timeout -k 10 300 python -u profiles/dc_probe.py 3 skew,linux,linuxwide,linux400 0,3 > gpurun_out/w3_dc.jsonl 2> gpurun_out/w3_dc.err
for k in 1 2; do
timeout -k 10 200 python -u bench.py --steps 20 --no-cpu --no-extras > gpurun_out/w3_bench_fused$k.json 2> gpurun_out/w3_bench_fused$k.err
timeout -k 10 200 python -u bench.py --steps 20 --no-cpu --no-extras --join-side > gpurun_out/w3_bench_side$k.json 2> gpurun_out/w3_bench_side$k.err
done
