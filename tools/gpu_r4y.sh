# round 4 final checks on the shipped build: the whole GPU suite, smoke, and the 200:55 bench line (prep change)
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4y; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/gtest.log 2>&1 || { tail -30 $O/gtest.log; exit 1; }
tail -1 $O/gtest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
cat $O/smoke.log
timeout -k 10 400 python bench.py --config 200:55 --steps 5 > $O/bench_20055.json 2> $O/bench_20055.err || exit 1
cut -c1-400 $O/bench_20055.json
