#!/bin/bash
# Resident-worker check after a change: single calls, the worker + parity + pipeline GPU tests, latency (x2).
set -o pipefail
out=gpurun_out/worker2; mkdir -p $out
for q in d de eed; do timeout -k 5 20 ./tools/worker_check 20 23 1440 3 $q > /dev/null || exit 1; done
timeout -k 5 20 ./tools/worker_check 2 3 16 1 ede > /dev/null || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_worker.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $out/gtest.log 2>&1 || { tail -40 $out/gtest.log; exit 1; }
tail -1 $out/gtest.log
for i in 1 2; do timeout -k 10 90 ./tools/latency_bench > $out/lat$i.json 2>&1 || { cat $out/lat$i.json; exit 1; }
  python3 -c "import json; d=json.load(open('$out/lat$i.json')); print({k: round(v,2) for k,v in d.items() if k.endswith('_us') and ('kfec_' in k or 'ping' in k) and 'flush' not in k})"; done
