#!/bin/bash
# PMC passes for the dominant kernel (vertex emission).  Counters are collected
# in separate rocprofv3 runs (kernel trace only, no sys/runtime trace), per
# MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE in separate passes.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${1:-gpurun_out/pmc}
K=${2:-k_vtx_pairs}
ARGS="python3 bench.py --steps 2 --warmup 1 --no-cpu"
rocprofv3 --kernel-include-regex "$K" --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- $ARGS > $OUT.fetch.log 2>&1
rocprofv3 --kernel-include-regex "$K" --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- $ARGS > $OUT.write.log 2>&1
rocprofv3 --kernel-include-regex "$K" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/sq -o run -- $ARGS > $OUT.sq.log 2>&1
rocprofv3 --kernel-include-regex "$K" --pmc SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/sq2 -o run -- $ARGS > $OUT.sq2.log 2>&1
