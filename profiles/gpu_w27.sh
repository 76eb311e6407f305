#!/bin/bash
# r05: k_match staging with plain loads instead of non-temporal ones (8 and 12 words per batch;
# profiles/ab_plain, ab_plain12) against HEAD (profiles/ab_head), alternated
set -e -o pipefail
mkdir -p gpurun_out/w27
for k in 1 2; do
  for V in head plain plain12; do
    WG_PKG_DIR=$PWD/profiles/ab_$V timeout -k 10 300 python -u profiles/match_probe.py > gpurun_out/w27/${V}_$k.jsonl 2> gpurun_out/w27/${V}_$k.err
  done
done
