set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_frames.py tests/test_gpu_parity.py > gpurun_out/r06bk_tests.log 2>&1 &&
timeout -k 10 200 profiles/emit_modes.sh r06bk 10 4 place4 &&
timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/r06bk_bench.json 2> gpurun_out/r06bk_bench.err
