# what the driver runs at round end, on the GPU box: smoke() then the default bench line (CPU leg included)
set -e -o pipefail
OUT=gpurun_out/${1:-driver}
mkdir -p $OUT
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1
timeout -k 10 600 python -u bench.py > $OUT/bench.json 2> $OUT/bench.err
