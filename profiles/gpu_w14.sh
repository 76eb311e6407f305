#!/bin/bash
# r05: randomised malformed lists through the speculative / deferred paths
set -e -o pipefail
mkdir -p gpurun_out/w14
timeout -k 10 600 python -u -m pytest tests/test_gpu_malformed.py -x -v --timeout 500 --timeout-method thread > gpurun_out/w14/malformed.log 2>&1
