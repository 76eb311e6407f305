#!/bin/bash
# r05: byte-parallel k_match — search + frames parity, then the 1M-row search leg
set -e -o pipefail
mkdir -p gpurun_out/w10
timeout -k 10 400 python -u -m pytest tests/test_gpu_search.py -x -v --timeout 200 --timeout-method thread > gpurun_out/w10/search_tests.log 2>&1
timeout -k 10 300 python -u profiles/match_probe.py > gpurun_out/w10/match_probe.jsonl 2> gpurun_out/w10/match_probe.err
timeout -k 10 300 python -u -m pytest tests/test_gpu_frames.py -x -q --timeout 200 --timeout-method thread > gpurun_out/w10/frames_tests.log 2>&1
