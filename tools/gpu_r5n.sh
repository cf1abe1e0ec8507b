#!/bin/bash
# Round 5, final queue numbers: sealed deferred delay against the flush size (tools/gpu_r5j.sh) and the per-call /
# queue latency record -- worker path three times, the queues' launch path (KFEC_QUEUE_WORKER_MAX=0) once.
set -o pipefail
bash tools/gpu_r5j.sh || exit 1
out=gpurun_out/r5n; mkdir -p $out
for i in 1 2 3; do timeout -k 10 90 ./tools/latency_bench > $out/latency_$i.json 2>&1 || { cat $out/latency_$i.json; exit 1; }; done
KFEC_QUEUE_WORKER_MAX=0 timeout -k 10 90 ./tools/latency_bench > $out/latency_launchq.json 2>&1 || { cat $out/latency_launchq.json; exit 1; }
for f in $out/latency_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', {k: round(v,2) for k,v in d.items() if k.endswith('_us') and 'p90' not in k})"; done
echo done
