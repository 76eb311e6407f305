set -e -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pe
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-include-regex k_vtx_tile --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/pe/f -o run -- python3 $R/profiles/emulate_shards.py --world 2 --steps 2 > $R/gpurun_out/pe/f.json 2> $R/gpurun_out/pe/f.err
timeout -s KILL 240 rocprofv3 --kernel-include-regex k_vtx_tile --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/pe/w -o run -- python3 $R/profiles/emulate_shards.py --world 2 --steps 2 > $R/gpurun_out/pe/w.json 2> $R/gpurun_out/pe/w.err
timeout -s KILL 240 rocprofv3 --kernel-include-regex k_vtx_tile --pmc TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum --output-format csv -d $R/gpurun_out/pe/t -o run -- python3 $R/profiles/emulate_shards.py --world 2 --steps 2 > $R/gpurun_out/pe/t.json 2> $R/gpurun_out/pe/t.err
