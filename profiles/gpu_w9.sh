#!/bin/bash
# r05: the emission's read folded into k_vtx_prep — parity + A/B (wide16 1M, C3)
set -e -o pipefail
mkdir -p gpurun_out/w9
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_spec.py tests/test_gpu_frames.py tests/test_gpu_shard.py tests/test_gpu_c5.py -x -q --timeout 300 --timeout-method thread > gpurun_out/w9/tests.log 2>&1
for k in 1 2 3; do
  timeout -k 10 200 python -u bench.py --steps 20 --no-cpu --no-extras > gpurun_out/w9/fused_$k.json 2> gpurun_out/w9/fused_$k.err
  timeout -k 10 200 python -u bench.py --steps 20 --no-cpu --no-extras --no-fused-read > gpurun_out/w9/plain_$k.json 2> gpurun_out/w9/plain_$k.err
done
for k in 1 2; do
  timeout -k 10 200 python -u bench.py --steps 50 --no-cpu --no-extras --kind random13 --rows-per-gpu 100000 > gpurun_out/w9/c3fused_$k.json 2> gpurun_out/w9/c3fused_$k.err
  timeout -k 10 200 python -u bench.py --steps 50 --no-cpu --no-extras --kind random13 --rows-per-gpu 100000 --no-fused-read > gpurun_out/w9/c3plain_$k.json 2> gpurun_out/w9/c3plain_$k.err
done
