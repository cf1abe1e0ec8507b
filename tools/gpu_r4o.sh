# round 4: PCIe-inclusive end to end (pinned host memory in and out), 20:3 and 10:3
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4o; mkdir -p $O
timeout -k 10 300 python tools/e2e.py > $O/e2e_203.json 2> $O/e2e_203.err || { tail $O/e2e_203.err; exit 1; }
timeout -k 10 300 python tools/e2e.py --K 10 --R 3 --B 1400 > $O/e2e_103.json 2> $O/e2e_103.err || { tail $O/e2e_103.err; exit 1; }
cat $O/e2e_203.json $O/e2e_103.json
