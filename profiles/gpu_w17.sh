#!/bin/bash
# r05: atlas rebuilds reuse the parse — font tests, then the bench's C2 leg
set -e -o pipefail
mkdir -p gpurun_out/w17
timeout -k 10 300 python -u -m pytest tests/test_gpu_font.py tests/test_gpu_text.py -x -q --timeout 200 --timeout-method thread > gpurun_out/w17/tests.log 2>&1
timeout -k 10 400 python -u bench.py --steps 5 > gpurun_out/w17/bench.json 2> gpurun_out/w17/bench.err
