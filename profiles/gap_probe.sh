# where the step's idle gaps come from: traced steps with and without the
# bench's timing events (profiles/gaps.py on each), plus untraced step times
set -e -o pipefail
TAG=${1:-r03t}
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd "$ROOT"
for i in 1 2; do
timeout -k 10 200 python bench.py --no-cpu --no-extras --steps 20 --warmup 5 > $OUT/ev$i.json 2>> $OUT/err.log
timeout -k 10 200 python bench.py --no-cpu --no-extras --steps 20 --warmup 5 --no-events > $OUT/noev$i.json 2>> $OUT/err.log
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tr_ev" -o run -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu --no-extras > "$OUT/tr_ev.json" 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$OUT/tr_noev" -o run -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 --no-cpu --no-extras --no-events > "$OUT/tr_noev.json" 2>&1
