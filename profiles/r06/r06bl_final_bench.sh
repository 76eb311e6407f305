set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06bl_smoke.log 2>&1 &&
timeout -k 10 400 python -u bench.py > gpurun_out/r06bl_bench.json 2> gpurun_out/r06bl_bench.err
