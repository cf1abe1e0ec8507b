#!/bin/bash
# Round pass, part 1 (tests, smoke, bench lines with the CPU baseline, wire / seal / pipeline benches).
# Outputs under gpurun_out/round/; tools/collect_round.py copies the judged summaries into profiles/.
set -o pipefail
out=gpurun_out/round; mkdir -p $out
echo "affinity=$(python3 -c 'import os; print(len(os.sched_getaffinity(0)))') nproc=$(nproc) cpu.max=$(cat /sys/fs/cgroup/cpu.max 2>/dev/null)" > $out/box.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $out/gtest.log 2>&1 || { tail -30 $out/gtest.log; exit 1; }
tail -2 $out/gtest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { cat $out/smoke.log; exit 1; }
cat $out/smoke.log
timeout -k 10 300 python bench.py > $out/bench_203.json 2> $out/bench_203.err || exit 1
timeout -k 10 300 python bench.py --config 10:3dec > $out/bench_103dec.json 2> $out/bench_103dec.err || exit 1
timeout -k 10 400 python bench.py --config 200:55 --steps 5 > $out/bench_20055.json 2> $out/bench_20055.err || exit 1
timeout -k 10 300 python bench.py --config 20:3loss1 > $out/bench_203loss1.json 2> $out/bench_203loss1.err || exit 1
cut -c1-300 $out/bench_*.json
timeout -k 10 200 python tools/bench_wire.py > $out/wire.json || exit 1
timeout -k 10 200 python tools/bench_seal.py > $out/seal.json || exit 1
timeout -k 10 200 python tools/bench_wire.py --ragged > $out/wire_ragged.json || exit 1
for t in 1 2 4 8; do timeout -k 10 300 ./tools/pipeline_bench 20 23 1440 16384 4 3 $t || exit 1; done > $out/pipeline_threads.json
timeout -k 10 120 ./tools/latency_bench > $out/latency.json || exit 1
KFEC_WORKER=0 timeout -k 10 120 ./tools/latency_bench > $out/latency_launch.json || exit 1
timeout -k 10 120 ./tools/side_effects 400 > $out/side_effects.jsonl || exit 1
timeout -k 10 300 python tools/concurrent_bench.py > $out/concurrent.json || exit 1
for mode in none chacha20; do for G in 16 256 4096; do F=$(( G >= 4096 ? 5 : 33 )); PB_SEAL=$mode timeout -k 10 120 ./tools/pipeline_bench 20 23 1440 $G $F 3 1 || exit 1; done; done > $out/pipeline_sealed.jsonl
timeout -k 10 600 python tools/e2e.py > $out/e2e.json 2> $out/e2e.err || { tail $out/e2e.err; exit 1; }
echo round-done
