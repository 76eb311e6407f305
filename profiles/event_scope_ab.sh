# same-box A/B of the timing / fork-join event scope (device vs HIP's default system fence)
set -e -o pipefail
OUT=gpurun_out/${1:-r03s}
mkdir -p $OUT
for i in 1 2; do
timeout -k 10 200 python bench.py --no-cpu --no-extras --steps 20 --warmup 5 > $OUT/dev$i.json 2>> $OUT/err.log
WG_EVENT_SCOPE=system timeout -k 10 200 python bench.py --no-cpu --no-extras --steps 20 --warmup 5 > $OUT/sys$i.json 2>> $OUT/err.log
done
