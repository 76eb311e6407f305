set -e -o pipefail
OUT=gpurun_out/r03l
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/t.log 2>&1
timeout -k 10 300 python profiles/tune_replay.py --kind wide16 --chunks auto,512:0,128:256,128:512,64:256,64:512,128:128,192:256 > $OUT/tune_wide16.jsonl 2> $OUT/tune.err
timeout -k 10 300 python profiles/tune_replay.py --kind random13 --rows 100000 --chunks auto,256:256,128:256,128:512,64:256,64:512,128:128,64:128 > $OUT/tune_r13.jsonl 2>> $OUT/tune.err
timeout -k 10 300 python profiles/tune_replay.py --kind linux --rows 1300000 --chunks auto,512:0,256:256 > $OUT/tune_linux.jsonl 2>> $OUT/tune.err
timeout -k 10 240 python bench.py --no-cpu > $OUT/bench.json 2> $OUT/bench.err
timeout -k 10 400 python profiles/emulate_shards.py --world 8 --steps 3 --out $OUT/emu8.json > $OUT/emu8.log 2>&1
timeout -k 10 400 python profiles/emulate_shards.py --world 8 --steps 3 --two-calls --out $OUT/emu8_two.json > $OUT/emu8_two.log 2>&1
