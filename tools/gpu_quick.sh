#!/bin/bash
# Quick GPU pass during development: GPU tests, then one bench line per config (no CPU leg).
# Outputs under gpurun_out/quick/.
set -o pipefail
out=gpurun_out/quick; mkdir -p $out
echo "affinity=$(python3 -c 'import os; print(len(os.sched_getaffinity(0)))') nproc=$(nproc) cpu.max=$(cat /sys/fs/cgroup/cpu.max 2>/dev/null)" > $out/box.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $out/gtest.log 2>&1 || { tail -40 $out/gtest.log; exit 1; }
tail -2 $out/gtest.log
for cfg in ${CONFIGS:-20:3 10:3dec 20:3loss1 200:55}; do
  steps=20; [ "$cfg" = "200:55" ] && steps=5
  timeout -k 10 300 python bench.py --config $cfg --no-cpu --steps $steps --warmup 2 > $out/bench_${cfg/:/_}.json 2> $out/bench_${cfg/:/_}.err || { cat $out/bench_${cfg/:/_}.err | tail -20; exit 1; }
  cut -c1-300 $out/bench_${cfg/:/_}.json
done
echo quick-done
