#!/bin/bash
# r05: k_match counters on the search probe (1M rows, four queries x 11 launches), one pass per group
set -e -o pipefail
OUT=gpurun_out/pmc_match
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
G1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"
G2="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_WR SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT"
G3="SQ_IFETCH SQ_INSTS_BRANCH SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA"
i=0
for G in "$G1" "$G2" "$G3"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-include-regex "k_match" --pmc $G --output-format csv -d $R/$OUT/g$i -o run -- python3 $R/profiles/match_probe.py > $R/$OUT/g$i.jsonl 2> $R/$OUT/g$i.err
done
