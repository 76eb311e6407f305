#!/bin/bash
# r05: emission tile A/B (1024 vs 2048) on C4, linuxwide, wide16 1M / 3M; the tile parity tests
set -e -o pipefail
mkdir -p gpurun_out/w6
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "tile_sizes or baseline_configs" -x -v --timeout 300 --timeout-method thread > gpurun_out/w6/tests.log 2>&1
for spec in "linux 1300000" "linuxwide 1000000" "wide16 1000000" "wide16 3000000"; do
  set -- $spec
  for t in 1024 2048; do
    timeout -k 10 200 python -u bench.py --steps 10 --no-cpu --no-extras --kind $1 --rows-per-gpu $2 --vtx-tile $t > gpurun_out/w6/$1_$2_$t.json 2> gpurun_out/w6/$1_$2_$t.err
  done
done
