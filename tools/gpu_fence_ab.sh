#!/bin/bash
# Per-call worker fence A/B: light fences (KFEC_WORKER_FENCES=1, no L2 invalidate / write-back per request) vs
# full system-scope acquire/release (=0); parity tests first (light is the default), then latency alternating.
set -o pipefail
out=gpurun_out/fence_ab; mkdir -p $out
for q in d de eed; do timeout -k 5 20 ./tools/worker_check 20 23 1440 3 $q > /dev/null || exit 1; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_worker.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $out/gtest.log 2>&1 || { tail -40 $out/gtest.log; exit 1; }
tail -1 $out/gtest.log
for i in 1 2; do
  for f in 0 1; do
    KFEC_WORKER_FENCES=$f timeout -k 10 90 ./tools/latency_bench > $out/lat_f${f}_$i.json 2>&1 || { cat $out/lat_f${f}_$i.json; exit 1; }
    python3 -c "import json; d=json.load(open('$out/lat_f${f}_$i.json')); print('FENCES=$f', {k: round(v,2) for k,v in d.items() if k.endswith('_us') and ('kfec_' in k or 'ping' in k) and 'flush' not in k and 'p90' not in k})"
  done
done
for f in 0 1; do
  KFEC_WORKER_FENCES=$f KFEC_WORKER_DEBUG=2 timeout -k 5 30 ./tools/worker_check 20 23 1440 3 $(printf "ed%.0s" {1..300}) > $out/phases_f$f.txt 2>&1 || { cat $out/phases_f$f.txt; exit 1; }
  echo "FENCES=$f"; tail -3 $out/phases_f$f.txt
done
