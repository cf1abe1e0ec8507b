#!/bin/bash
# BAR staging A/B for the per-call worker: latency with the request side in device memory written through the
# BAR (KFEC_WORKER_BAR=1) vs in the pinned host slot (=0), alternating, plus the device-side phase times of each.
set -o pipefail
out=gpurun_out/bar_ab; mkdir -p $out
for i in 1 2; do
  for b in 0 1; do
    KFEC_WORKER_BAR=$b timeout -k 10 90 ./tools/latency_bench > $out/lat_bar${b}_$i.json 2>&1 || { cat $out/lat_bar${b}_$i.json; exit 1; }
    python3 -c "import json; d=json.load(open('$out/lat_bar${b}_$i.json')); print('BAR=$b', {k: round(v,2) for k,v in d.items() if k.endswith('_us') and ('kfec_' in k or 'ping' in k) and 'flush' not in k})"
  done
done
for b in 0 1; do
  KFEC_WORKER_BAR=$b KFEC_WORKER_DEBUG=2 timeout -k 5 30 ./tools/worker_check 20 23 1440 3 $(printf "ed%.0s" {1..300}) > $out/phases_bar$b.txt 2>&1 || { cat $out/phases_bar$b.txt; exit 1; }
  echo "BAR=$b"; tail -4 $out/phases_bar$b.txt
done
