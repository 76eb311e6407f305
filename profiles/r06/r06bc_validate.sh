set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_frames.py tests/test_gpu_parity.py > gpurun_out/r06bc_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/r06bc_bench.json 2> gpurun_out/r06bc_bench.err &&
timeout -k 10 200 profiles/emit_modes.sh r06bc 10 4 place4
