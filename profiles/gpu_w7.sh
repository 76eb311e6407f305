#!/bin/bash
set -e -o pipefail
mkdir -p gpurun_out/w7
for t in 2048 4096 2048 4096; do
  timeout -k 10 200 python -u bench.py --steps 10 --no-cpu --no-extras --kind linuxwide --vtx-tile $t > gpurun_out/w7/lw_$t.json 2> gpurun_out/w7/lw_$t.err
  timeout -k 10 200 python -u bench.py --steps 10 --no-cpu --no-extras --kind wide16 --rows-per-gpu 3000000 --vtx-tile $t > gpurun_out/w7/w3m_$t.json 2> gpurun_out/w7/w3m_$t.err
done
