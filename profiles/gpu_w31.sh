#!/bin/bash
# r05: k_probe_fix / k_lf_events first loads issued before their dup / gate checks (main tree) against
# HEAD (profiles/ab_head), bench alternated twice; then the GPU suite on the main tree
set -e -o pipefail
mkdir -p gpurun_out/w31
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/w31/a_$k.json 2> gpurun_out/w31/a_$k.err
  WG_PKG_DIR=$PWD/profiles/ab_head timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/w31/head_$k.json 2> gpurun_out/w31/head_$k.err
done
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/w31/tests.log 2>&1
