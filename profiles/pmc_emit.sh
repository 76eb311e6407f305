#!/bin/bash
# SQ counters of k_vtx_tile on two workloads (wide16 1M, linux 1.3M), one
# counter group per rocprofv3 pass, kernel trace only (never with sys/runtime
# traces).  Output under gpurun_out/pmc_emit/<group>_<work>/.
set -e -o pipefail
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_emit
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"
G2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT"
for w in wide16:1000000 linux:1300000; do
  n=${w%%:*}
  i=1
  for g in "$G1" "$G2"; do
    timeout -s KILL 120 rocprofv3 --kernel-include-regex k_vtx_tile --pmc $g --output-format csv -d "$OUT/g${i}_$n" -o run -- python3 $ROOT/profiles/emit_variants.py --work $w --steps 3 > "$OUT/g${i}_$n.log" 2>&1
    i=$((i+1))
  done
done
