#!/bin/bash
# Round 3 session check: resident-worker latency (worker vs launch path), worker + parity GPU tests,
# and the small-K persistent syndrome decode A/B (ss0 = syn_kernel + per-item expand loads, ss1 = syn_small_kernel + batched expand) at 10:3 random and 200:55.
set -o pipefail
out=gpurun_out/r3a; mkdir -p $out
for q in d de eed; do timeout -k 5 20 ./tools/worker_check 20 23 1440 3 $q || exit 1; done
timeout -k 10 90 ./tools/latency_bench > $out/latency.json 2>&1 || { cat $out/latency.json; exit 1; }
cat $out/latency.json
KFEC_WORKER=0 timeout -k 10 90 ./tools/latency_bench > $out/latency_launch.json 2>&1 || { cat $out/latency_launch.json; exit 1; }
cat $out/latency_launch.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_worker.py tests/test_gpu_parity.py -x -v --timeout 120 --timeout-method thread > $out/gtest.log 2>&1 || { tail -40 $out/gtest.log; exit 1; }
tail -2 $out/gtest.log
V=kcptube_amd/variants
AB_ERASE=random timeout -k 10 400 python tools/ab.py 3 $V/libkfec_ss0.so $V/libkfec_ss1.so -- 10 13 1400 1048576 > $out/ab_103.txt 2>&1 || { cat $out/ab_103.txt; exit 1; }
cat $out/ab_103.txt
timeout -k 10 600 python tools/ab.py 2 $V/libkfec_ss0.so $V/libkfec_ss1.so -- 200 255 1440 65536 > $out/ab_20055.txt 2>&1 || { cat $out/ab_20055.txt; exit 1; }
cat $out/ab_20055.txt
