#!/bin/bash
# r05: k_match occupancy A/B in one call: main tree (8 staged words, 4 waves/SIMD) against
# builds at 5 waves/SIMD with 2 / 4 / 8 staged words (profiles/ab_sb*o5), alternated
set -e -o pipefail
mkdir -p gpurun_out/w21
for k in 1 2; do
  timeout -k 10 300 python -u profiles/match_probe.py > gpurun_out/w21/base_$k.jsonl 2> gpurun_out/w21/base_$k.err
  for V in sb4o5 sb2o5 sb8o5; do
    WG_PKG_DIR=$PWD/profiles/ab_$V timeout -k 10 300 python -u profiles/match_probe.py > gpurun_out/w21/${V}_$k.jsonl 2> gpurun_out/w21/${V}_$k.err
  done
done
