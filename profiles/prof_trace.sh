set -e -o pipefail
ROOT=$GRAFT_REPO_ROOT
OUT=$ROOT/gpurun_out/p1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/main -o run -- python3 $ROOT/bench.py --steps 3 --warmup 1 --no-cpu --no-extras > $OUT/main.json 2> $OUT/main.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/extra -o run -- python3 $ROOT/bench.py --steps 2 --warmup 1 --no-cpu > $OUT/extra.json 2> $OUT/extra.err
