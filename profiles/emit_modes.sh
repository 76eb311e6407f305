#!/bin/bash
# The emission's two rates against the GPU's clocks and power: a sampler of
# rocm-smi (its own process; reads only) beside an emission-only time series
# (profiles/emit_modes.py), run from the repo root:
#   profiles/emit_modes.sh <tag> [seconds] [engines] [placeK|realloc]   -> gpurun_out/<tag>_emit_series.jsonl, <tag>_smi.jsonl
set -e -o pipefail
TAG=${1:?tag}; SECS=${2:-30}; ENG=${3:-1}; MODE=${4:-}
mkdir -p gpurun_out
( end=$(( $(date +%s) + SECS + 90 ))
  while [ "$(date +%s)" -lt "$end" ]; do
    printf '{"t_unix": %s, "smi": ' "$(date +%s.%N)"
    timeout -k 5 10 rocm-smi --showpower --showclocks --showtemp --json 2>/dev/null | tr -d '\n' || printf 'null'
    printf '}\n'
    sleep 0.5
  done ) > "gpurun_out/${TAG}_smi.jsonl" &
SAMPLER=$!
timeout -k 10 240 python -u profiles/emit_modes.py "$SECS" "$ENG" $MODE > "gpurun_out/${TAG}_emit_series.jsonl" 2> "gpurun_out/${TAG}_emit_series.err"
kill "$SAMPLER" 2>/dev/null || true
wait "$SAMPLER" 2>/dev/null || true
