#!/bin/bash
# sharded-step emulation on one GPU: world 4 and 8 (wide16), and a kernel
# trace of the world-8 run -> gpurun_out/<tag>_*
set -e -o pipefail
TAG=${1:?tag}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u profiles/emulate_shards.py --world 4 --steps 3 --out $OUT/${TAG}_emu_w4.json > $OUT/${TAG}_emu_w4.log 2>&1
timeout -k 10 300 python -u profiles/emulate_shards.py --world 8 --steps 3 --out $OUT/${TAG}_emu_w8.json > $OUT/${TAG}_emu_w8.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/${TAG}_emutrace -o run -- python3 $R/profiles/emulate_shards.py --world 8 --steps 2 --out $OUT/${TAG}_emutrace.json > $OUT/${TAG}_emutrace.log 2>&1
