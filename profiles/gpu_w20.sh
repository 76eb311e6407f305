#!/bin/bash
# r05: k_match phase breakdown: the main tree against builds with one or more phases compiled out
# (WG_MATCH_SKIP bits: 1 Final_Sigma, 2 lowering, 4 first-byte match, 8 walks, 16 lead lists); timing only
set -e -o pipefail
mkdir -p gpurun_out/w20
for k in 1 2; do
  timeout -k 10 300 python -u profiles/match_probe.py > gpurun_out/w20/base_$k.jsonl 2> gpurun_out/w20/base_$k.err
  for S in 32 1 2 19; do
    WG_PKG_DIR=$PWD/profiles/ab_s$S timeout -k 10 300 python -u profiles/match_probe.py > gpurun_out/w20/s${S}_$k.jsonl 2> gpurun_out/w20/s${S}_$k.err
  done
done
