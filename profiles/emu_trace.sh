# kernel trace of the 8-rank shard emulation (per-segment kernels and gaps)
set -e -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-emutrace}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 $R/profiles/emulate_shards.py --world 8 --steps 2 --out $OUT/emu.json > $OUT/emu.log 2>&1
