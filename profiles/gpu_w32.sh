#!/bin/bash
# r05: the whole bench (baseline configs included) at HEAD against the session's starting build
# 532a8ea (profiles/ab_old), alternated twice: is linuxwide's 13.8 ms (r05w) a regression or the box?
set -e -o pipefail
mkdir -p gpurun_out/w32
for k in 1 2; do
  timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/w32/head_$k.json 2> gpurun_out/w32/head_$k.err
  WG_PKG_DIR=$PWD/profiles/ab_old timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/w32/old_$k.json 2> gpurun_out/w32/old_$k.err
done
