#!/bin/bash
# PMC passes for the non-emission kernels of a step:
# HBM traffic (FETCH_SIZE, WRITE_SIZE in separate passes), L2 hit rate and SQ
# instruction / wait counters, each pass a run of its own with kernel trace
# only (MI355X_MICROARCH.md §HBM; no sys/runtime traces beside --pmc).
#   profiles/pmc_step.sh r03a     (on the GPU box, from the repo root)
# -> gpurun_out/pmc_step_<tag>/{fetch,write,tcc,sq}/..., then
#    python3 profiles/pmc_step_summary.py gpurun_out/pmc_step_<tag> > profiles/<tag>_pmc_step.md
set -e -o pipefail
TAG=${1:-r03a}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/pmc_step_$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
RX=${PMC_KERNELS:-"k_probe_near|k_probe_fix|k_hash_place|k_hash_settle|k_lf_rows|k_lf_jump_tile|k_lf_replay|k_dc_iter|k_rt_walk|k_edges_rows|k_edge_counts|k_geom_offsets|k_top_carry|k_top_finish|k_sweep|k_curves_tb|k_curves|k_vtx_prep|k_vtx_tile"}
# (PMC_BENCH_ARGS: another config, e.g. "--kind linux --rows-per-gpu 1300000" for C4)
BENCH="$ROOT/bench.py --steps 3 --warmup ${PMC_WARMUP:-1} --no-cpu --no-extras ${PMC_BENCH_ARGS:-}"
timeout -s KILL 120 rocprofv3 --kernel-include-regex "$RX" --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 $BENCH > "$OUT/fetch.json" 2> "$OUT/fetch.err"
timeout -s KILL 120 rocprofv3 --kernel-include-regex "$RX" --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 $BENCH > "$OUT/write.json" 2> "$OUT/write.err"
timeout -s KILL 120 rocprofv3 --kernel-include-regex "$RX" --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$OUT/tcc" -o run -- python3 $BENCH > "$OUT/tcc.json" 2> "$OUT/tcc.err"
timeout -s KILL 120 rocprofv3 --kernel-include-regex "$RX" --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --output-format csv -d "$OUT/sq" -o run -- python3 $BENCH > "$OUT/sq.json" 2> "$OUT/sq.err"
python3 "$ROOT/profiles/pmc_step_summary.py" "$OUT" > "$OUT/summary.md"
