#!/bin/bash
# r05: capacity guards in one round trip reading the overflow word for absent pointers (main tree),
# HEAD (profiles/ab_head) and the first version with a __device__ zero array (profiles/ab_a1), alternated
set -e -o pipefail
mkdir -p gpurun_out/w29
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/w29/a2_$k.json 2> gpurun_out/w29/a2_$k.err
  WG_PKG_DIR=$PWD/profiles/ab_head timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/w29/head_$k.json 2> gpurun_out/w29/head_$k.err
  WG_PKG_DIR=$PWD/profiles/ab_a1 timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/w29/a1_$k.json 2> gpurun_out/w29/a1_$k.err
done
