#!/bin/bash
# the whole GPU suite as the driver runs it, plus the C++ mirror and smoke()
set -e -o pipefail
TAG=${1:-full}
mkdir -p gpurun_out
timeout -k 10 120 tests/cpp/test_graph_layout > gpurun_out/${TAG}_cxx.log 2>&1
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/${TAG}_smoke.log 2>&1
