# bench.py's N>1 path rehearsed on one GPU: gloo process group, every rank on cuda:0
set -e -o pipefail
OUT=gpurun_out/${1:-rehearse}
mkdir -p $OUT
for n in 2 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n --master-addr 127.0.0.1 --master-port $((29500 + n)) \
    bench.py --gpus $n --steps 5 --warmup 2 --dist-backend gloo --same-device --no-cpu --no-extras > $OUT/weak$n.json 2> $OUT/weak$n.err
done
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29509 \
  bench.py --gpus 4 --steps 5 --warmup 2 --dist-backend gloo --same-device --no-cpu --no-extras --total-rows 1000000 > $OUT/strong4.json 2> $OUT/strong4.err
