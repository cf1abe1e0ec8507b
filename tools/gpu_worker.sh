#!/bin/bash
# Resident-worker check: single calls (worker_check), device-side phase times, latency (worker vs launch path)
# and the worker + parity GPU tests.  Outputs under gpurun_out/worker/.
set -o pipefail
out=gpurun_out/worker; mkdir -p $out
for q in d de eed; do timeout -k 5 20 ./tools/worker_check 20 23 1440 3 $q || exit 1; done
timeout -k 5 20 ./tools/worker_check 2 3 16 1 ede || exit 1
KFEC_WORKER_DEBUG=2 timeout -k 10 90 ./tools/latency_bench > $out/latency_dbg.json 2>&1 || { cat $out/latency_dbg.json; exit 1; }
cat $out/latency_dbg.json
for wg in 2 4 8; do
  KFEC_WORKER_WGS=$wg timeout -k 10 90 ./tools/latency_bench > $out/latency_w$wg.json 2>&1 || { cat $out/latency_w$wg.json; exit 1; }
  cut -c1-200 $out/latency_w$wg.json
done
KFEC_WORKER=0 timeout -k 10 90 ./tools/latency_bench > $out/latency_launch.json 2>&1 || { cat $out/latency_launch.json; exit 1; }
cut -c1-200 $out/latency_launch.json
timeout -k 10 600 python -u -m pytest tests/test_gpu_worker.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $out/gtest.log 2>&1 || { tail -40 $out/gtest.log; exit 1; }
tail -2 $out/gtest.log
