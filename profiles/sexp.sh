set -e -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/sexp
cd /tmp && export TMPDIR=/tmp
for v in base nofill noloop; do
  L=$R/whisper-git_amd/wgraph/libwgraph.so
  [ $v != base ] && L=$R/whisper-git_amd/wgraph/libwgraph_$v.so
  WGRAPH_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/sexp/$v -o run -- python3 $R/profiles/search_probe.py > $R/gpurun_out/sexp/$v.txt 2>&1
done
