set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_spec.py tests/test_gpu_frames.py tests/test_gpu_c5.py > gpurun_out/r06bh_tests.log 2>&1 &&
bash profiles/ab_lib.sh r06bh ab/lib_base.so ab/lib_sweep.so 3
