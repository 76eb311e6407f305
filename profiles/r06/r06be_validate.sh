set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_frames.py > gpurun_out/r06be_frames.log 2>&1 &&
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r06be_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06be_smoke.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/r06be_bench.json 2> gpurun_out/r06be_bench.err
