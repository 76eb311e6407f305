#!/bin/bash
# r05: sharded tests, C5, frames, the C++ mirror, the 8-rank emulation (wide16, skew), the default bench
set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 tests/cpp/test_graph_layout > gpurun_out/w4_cxx.log 2>&1
timeout -k 10 700 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_c5.py tests/test_gpu_frames.py -x -v --timeout 300 --timeout-method thread > gpurun_out/w4_tests.log 2>&1
timeout -k 10 300 python -u profiles/emulate_shards.py --world 8 --steps 3 --kind skew --out gpurun_out/w4_emu_skew.json > gpurun_out/w4_emu_skew.log 2>&1
timeout -k 10 300 python -u profiles/emulate_shards.py --world 8 --steps 3 --out gpurun_out/w4_emu_wide16.json > gpurun_out/w4_emu_wide16.log 2>&1
timeout -k 10 400 python -u bench.py > gpurun_out/w4_bench.json 2> gpurun_out/w4_bench.err
