#!/bin/bash
# r05: k_match's local walks read by words with one in flight (main tree) against HEAD (profiles/ab_head),
# alternated three times; then the search tests
set -e -o pipefail
mkdir -p gpurun_out/w33
for k in 1 2 3; do
  timeout -k 10 300 python -u profiles/match_probe.py > gpurun_out/w33/a_$k.jsonl 2> gpurun_out/w33/a_$k.err
  WG_PKG_DIR=$PWD/profiles/ab_head timeout -k 10 300 python -u profiles/match_probe.py > gpurun_out/w33/b_$k.jsonl 2> gpurun_out/w33/b_$k.err
done
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_search.py > gpurun_out/w33/search_tests.log 2>&1
