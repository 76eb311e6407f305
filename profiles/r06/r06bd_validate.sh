set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_text.py tests/test_gpu_frames.py > gpurun_out/r06bd_tests.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu > gpurun_out/r06bd_bench.json 2> gpurun_out/r06bd_bench.err
