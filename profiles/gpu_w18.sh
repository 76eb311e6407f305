#!/bin/bash
# r05: k_match staging batch A/B in one call (A = main tree, B = profiles/ab_pkg copy), alternated
set -e -o pipefail
mkdir -p gpurun_out/w18
for k in 1 2 3; do
  timeout -k 10 300 python -u profiles/match_probe.py > gpurun_out/w18/a_$k.jsonl 2> gpurun_out/w18/a_$k.err
  WG_PKG_DIR=$PWD/profiles/ab_pkg timeout -k 10 300 python -u profiles/match_probe.py > gpurun_out/w18/b_$k.jsonl 2> gpurun_out/w18/b_$k.err
done
