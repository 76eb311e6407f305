#!/bin/bash
set -e -o pipefail
mkdir -p gpurun_out/w8
timeout -k 10 300 python -u -m pytest tests/test_gpu_search.py -x -q --timeout 300 --timeout-method thread > gpurun_out/w8/search_tests.log 2>&1
timeout -k 10 300 python -u profiles/match_probe.py > gpurun_out/w8/match.jsonl 2> gpurun_out/w8/match.err
timeout -k 10 300 python -u profiles/pipeline_probe.py 20 > gpurun_out/w8/pipe.log 2>&1
