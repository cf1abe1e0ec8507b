#!/bin/bash
# Per-call worker: latency against the number of resident workgroups (KFEC_WORKER_WGS), BAR staging on.
set -o pipefail
out=gpurun_out/wgs; mkdir -p $out
for r in 1 2; do for w in 2 4 8; do
  KFEC_WORKER_WGS=$w timeout -k 10 90 ./tools/latency_bench > $out/lat_w${w}_$r.json 2>&1 || { cat $out/lat_w${w}_$r.json; exit 1; }
  python3 -c "import json; d=json.load(open('$out/lat_w${w}_$r.json')); print('WGS=$w', {k: round(v,2) for k,v in d.items() if k.endswith('_us') and ('kfec_' in k or 'ping' in k) and 'flush' not in k and 'p90' not in k and 'p50' not in k})"
done; done
