#!/bin/bash
# Round 5 baseline: queue-flush latency and sealed deferred delay on the round-4 code.
set -o pipefail
out=gpurun_out/r5a; mkdir -p $out
timeout -k 10 120 ./tools/latency_bench > $out/latency.json 2>&1 || { cat $out/latency.json; exit 1; }
for mode in none chacha20; do PB_SEAL=$mode timeout -k 10 120 ./tools/pipeline_bench 20 23 1440 16 33 3 1 || exit 1; done > $out/sealed16.jsonl
cat $out/latency.json; cut -c1-200 $out/sealed16.jsonl
