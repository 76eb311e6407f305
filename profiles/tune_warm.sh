set -e -o pipefail
mkdir -p gpurun_out/r03w
timeout -k 10 250 python profiles/tune_replay.py --kind wide16 --chunks 128:512,128:384,128:448,192:384,192:512,128:640 > gpurun_out/r03w/tune.jsonl 2> gpurun_out/r03w/tune.err
timeout -k 10 250 python profiles/tune_replay.py --kind wide16 --chunks 128:640,128:448,128:512 >> gpurun_out/r03w/tune.jsonl 2>> gpurun_out/r03w/tune.err
