# global replay chunk / warm-up in the 8-rank emulation (kernel traces)
set -e -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-emutune}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in auto 128:512 128:256 128:128 256:256 256:512 64:256; do
  tag=${v/:/_}
  extra=""
  [ $v != auto ] && extra="--replay $v"
  timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/$tag -o run -- python3 $R/profiles/emulate_shards.py --world 8 --steps 3 $extra --out $OUT/$tag.json > $OUT/$tag.log 2>&1
done
