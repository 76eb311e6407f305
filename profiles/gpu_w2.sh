set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_replay_forms.py tests/test_gpu_lanes_wide.py tests/test_lane_pins.py tests/test_gpu_spec.py -x -v --timeout 300 --timeout-method thread > gpurun_out/w2_tests.log 2>&1
timeout -k 10 300 python -u profiles/dc_probe.py 3 skew,linux,linuxwide,linux400 0,3 > gpurun_out/w2_dc.jsonl 2> gpurun_out/w2_dc.err
