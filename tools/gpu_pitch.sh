#!/bin/bash
# Shard-pitch A/B: kernel times at the packed pitch vs line-aligned pitches, bench lines at
# pitch = B and pitch = 1536, and the PMC passes of both 20:3 layouts.  Outputs under gpurun_out/pitch/.
set -o pipefail
out=gpurun_out/pitch; mkdir -p $out
timeout -k 10 300 python tools/pitch_ab.py 3 1440 1472 1536 > $out/ab_203.txt 2>&1 || { tail $out/ab_203.txt; exit 1; }
PITCH_AB_CFG=10:13:1400:random timeout -k 10 300 python tools/pitch_ab.py 3 1400 1408 1536 > $out/ab_103.txt 2>&1 || { tail $out/ab_103.txt; exit 1; }
timeout -k 10 300 python bench.py --no-cpu > $out/bench_203.json 2> $out/bench_203.err || exit 1
timeout -k 10 300 python bench.py --no-cpu --pitch 1536 > $out/bench_203_p1536.json 2> $out/bench_203_p1536.err || exit 1
timeout -k 10 300 python bench.py --no-cpu --config 10:3dec --pitch 1536 > $out/bench_103dec_p1536.json 2> $out/bench_103dec_p1536.err || exit 1
bash tools/profile.sh r03_203_p1536 --steps 5 --warmup 1 --no-cpu --pitch 1536 || exit 1
bash tools/profile.sh r03_203 --steps 5 --warmup 1 --no-cpu || exit 1
echo pitch-done
