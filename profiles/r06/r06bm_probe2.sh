set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py --no-cpu --no-extras --steps 30 > gpurun_out/r06bm_bench.json 2> gpurun_out/r06bm_bench.err &&
timeout -k 10 200 profiles/emit_modes.sh r06bm 10 8 place4
