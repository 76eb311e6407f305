#!/bin/bash
# r05: k_match lead lists written after all staging loads (one scan per wave) with 8 / 16 / 24 staged
# words per thread and batch (profiles/ab_d8, ab_d16, ab_d24) against HEAD (profiles/ab_head), alternated
set -e -o pipefail
mkdir -p gpurun_out/w26
for k in 1 2; do
  for V in head d8 d16 d24; do
    WG_PKG_DIR=$PWD/profiles/ab_$V timeout -k 10 300 python -u profiles/match_probe.py > gpurun_out/w26/${V}_$k.jsonl 2> gpurun_out/w26/${V}_$k.err
  done
done
