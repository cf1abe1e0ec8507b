set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4h; mkdir -p $O
timeout -k 10 200 tools/ceiling > $O/ceiling.txt 2>&1 || { cat $O/ceiling.txt; exit 1; }
cat $O/ceiling.txt
