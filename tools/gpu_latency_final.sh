#!/bin/bash
# Per-call latency record: the worker path three times, the launch path once, the worker's device phases.
set -o pipefail
out=gpurun_out/latfinal; mkdir -p $out
for i in 1 2 3; do timeout -k 10 90 ./tools/latency_bench > $out/latency_$i.json 2>&1 || { cat $out/latency_$i.json; exit 1; }; done
KFEC_WORKER=0 timeout -k 10 90 ./tools/latency_bench > $out/latency_launch.json 2>&1 || { cat $out/latency_launch.json; exit 1; }
KFEC_WORKER_DEBUG=2 timeout -k 5 30 ./tools/worker_check 20 23 1440 3 $(printf "ed%.0s" {1..500}) > $out/phases.txt 2>&1 || { cat $out/phases.txt; exit 1; }
for f in $out/latency_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', {k: round(v,2) for k,v in d.items() if k.endswith('_us') and ('kfec_' in k or 'ping' in k) and 'flush' not in k})"; done
tail -3 $out/phases.txt
timeout -k 5 60 ./tools/bar_probe > $out/bar_probe.txt 2>&1 && cat $out/bar_probe.txt
