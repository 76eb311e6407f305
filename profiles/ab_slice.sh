set -e -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_spec.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_tests.log 2>&1
for v in a b c; do
  timeout -k 10 120 python bench.py --no-cpu --no-extras --steps 20 --slice > gpurun_out/ab_s_$v.json 2> gpurun_out/ab_s_$v.err
  timeout -k 10 120 python bench.py --no-cpu --no-extras --steps 20 > gpurun_out/ab_n_$v.json 2> gpurun_out/ab_n_$v.err
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/ab_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 5 --warmup 2 --no-cpu --no-extras > $GRAFT_REPO_ROOT/gpurun_out/ab_prof.json 2>&1
