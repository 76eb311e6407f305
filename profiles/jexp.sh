set -e -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/jexp
for j in 0 2 3 4 8; do
  L=$R/whisper-git_amd/wgraph/libwgraph.so
  [ $j != 0 ] && L=$R/whisper-git_amd/wgraph/libwgraph_j$j.so
  WGRAPH_LIB=$L timeout -k 10 120 python3 $R/profiles/tune_replay.py --chunks 512 > $R/gpurun_out/jexp/w$j.txt 2>/dev/null
  WGRAPH_LIB=$L timeout -k 10 120 python3 $R/profiles/tune_replay.py --kind linux --rows 1300000 --chunks 512 > $R/gpurun_out/jexp/l$j.txt 2>/dev/null
done
