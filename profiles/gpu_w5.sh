#!/bin/bash
# r05: kernel traces of the bench step on wide16 (1M), linuxwide (1M), C3 (random13 100k), skew (1M)
set -e -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/w5
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for spec in "wide16 1000000" "linuxwide 1000000" "random13 100000" "skew 1000000"; do
  set -- $spec
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$1 -o run -- python3 $ROOT/bench.py --steps 5 --warmup 2 --no-cpu --no-extras --kind $1 --rows-per-gpu $2 > $OUT/$1.json 2> $OUT/$1.err
done
