set -e -o pipefail
ROOT=$GRAFT_REPO_ROOT
OUT=$ROOT/gpurun_out/pmc_side
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-include-regex "k_match|k_text_rows|k_vtx_tile" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES --output-format csv -d $OUT/a -o run -- python3 $ROOT/bench.py --steps 1 --warmup 0 --no-cpu > $OUT/a.json 2> $OUT/a.err
