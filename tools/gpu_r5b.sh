#!/bin/bash
# Round 5: queue paths (worker batch flushes), retry-safety, worker / side-effect tests, latency.
set -o pipefail
out=gpurun_out/r5b; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_queue_paths.py tests/test_gpu_pipeline.py -x -v --timeout 120 --timeout-method thread > $out/t1.log 2>&1 || { tail -40 $out/t1.log; exit 1; }
tail -3 $out/t1.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_worker.py tests/test_gpu_side_effects.py -x -v --timeout 120 --timeout-method thread > $out/t2.log 2>&1 || { tail -40 $out/t2.log; exit 1; }
tail -3 $out/t2.log
timeout -k 10 120 ./tools/latency_bench > $out/latency.json 2>&1 || { cat $out/latency.json; exit 1; }
KFEC_QUEUE_WORKER_MAX=0 timeout -k 10 120 ./tools/latency_bench > $out/latency_launchq.json 2>&1 || { cat $out/latency_launchq.json; exit 1; }
for mode in none chacha20; do PB_SEAL=$mode timeout -k 10 120 ./tools/pipeline_bench 20 23 1440 16 33 3 1 || exit 1; done > $out/sealed16.jsonl
timeout -k 10 300 ./tools/pipeline_bench 20 23 1440 16384 4 3 1 > $out/pipe16k.json || exit 1
cat $out/latency.json $out/latency_launchq.json; cut -c1-250 $out/sealed16.jsonl; cut -c1-400 $out/pipe16k.json
