#!/bin/bash
# Round-end style GPU pass: tests, smoke, bench lines for every config, rocprof summaries.  Outputs under
# gpurun_out/round/; tools/collect_round.py copies the judged summaries into profiles/.
set -o pipefail
out=gpurun_out/round; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $out/gtest.log 2>&1 || { tail -30 $out/gtest.log; exit 1; }
tail -2 $out/gtest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { cat $out/smoke.log; exit 1; }
cat $out/smoke.log
timeout -k 10 300 python bench.py > $out/bench_203.json 2> $out/bench_203.err || exit 1
timeout -k 10 200 python bench.py --config 10:3dec --no-cpu > $out/bench_103dec.json || exit 1
timeout -k 10 300 python bench.py --config 200:55 --no-cpu --steps 5 > $out/bench_20055.json || exit 1
cat $out/bench_*.json | cut -c1-400
timeout -k 10 200 python tools/bench_wire.py > $out/wire.json || exit 1
timeout -k 10 200 python tools/bench_seal.py > $out/seal.json || exit 1
timeout -k 10 200 python tools/bench_wire.py --ragged > $out/wire_ragged.json || exit 1
# host-memory pipeline (1..8 host threads) and the latency path; binaries built beforehand (tools/*.cpp headers)
for t in 1 2 4 8; do timeout -k 10 300 ./tools/pipeline_bench 20 23 1440 16384 4 3 $t || exit 1; done > $out/pipeline_threads.json
timeout -k 10 120 ./tools/latency_bench > $out/latency.json || exit 1
bash tools/gpu_profile_all.sh || exit 1
echo round-done
