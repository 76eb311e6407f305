# sharded path: the shard tests, then the 8-rank emulation with and without deferred validation
set -e -o pipefail
OUT=gpurun_out/${1:-r03x}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_shard.py tests/test_gpu_c5.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/t_shard.log 2>&1
timeout -k 10 400 python profiles/emulate_shards.py --world 8 --steps 3 --out $OUT/emu8.json > $OUT/emu8.log 2>&1
timeout -k 10 400 python profiles/emulate_shards.py --world 8 --steps 3 --no-defer --out $OUT/emu8_nodefer.json > $OUT/emu8_nodefer.log 2>&1
timeout -k 10 400 python profiles/emulate_shards.py --world 8 --steps 3 --no-spec-replay --out $OUT/emu8_nospec.json > $OUT/emu8_nospec.log 2>&1
