#!/bin/bash
# r05: geometry kernels' capacity guards read in one round trip (main tree) against HEAD's build
# (profiles/ab_head), bench alternated three times each; then the GPU suite on the main tree
set -e -o pipefail
mkdir -p gpurun_out/w28
for k in 1 2 3; do
  timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/w28/a_$k.json 2> gpurun_out/w28/a_$k.err
  WG_PKG_DIR=$PWD/profiles/ab_head timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/w28/b_$k.json 2> gpurun_out/w28/b_$k.err
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/w28/tests.log 2>&1
