set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests > gpurun_out/r06bn_gpu.log 2>&1 &&
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06bn_smoke.log 2>&1 &&
timeout -k 10 120 tests/cpp/test_graph_layout > gpurun_out/r06bn_cxx.log 2>&1
