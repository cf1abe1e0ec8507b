#!/bin/bash
# Round 5: adaptive BAR staging + sealed small flush; tests and latency / pipeline numbers.
set -o pipefail
out=gpurun_out/r5c; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_queue_paths.py tests/test_gpu_pipeline.py tests/test_gpu_frame.py -x -q --timeout 120 --timeout-method thread > $out/t1.log 2>&1 || { tail -40 $out/t1.log; exit 1; }
tail -3 $out/t1.log
timeout -k 10 120 ./tools/latency_bench > $out/latency.json 2>&1 || { cat $out/latency.json; exit 1; }
for mode in none chacha20 aes_gcm; do PB_SEAL=$mode timeout -k 10 120 ./tools/pipeline_bench 20 23 1440 16 33 3 1 || exit 1; done > $out/sealed16.jsonl
for G in 256 1024 4096 16384; do timeout -k 10 300 ./tools/pipeline_bench 20 23 1440 $G 4 3 1 || exit 1; done > $out/pipe.jsonl
for G in 256 1024 4096; do KFEC_QUEUE_BAR_MAX=0 timeout -k 10 300 ./tools/pipeline_bench 20 23 1440 $G 4 3 1 || exit 1; done > $out/pipe_dma.jsonl
for G in 256 1024; do KFEC_QUEUE_BAR_ALIGN=4 timeout -k 10 300 ./tools/pipeline_bench 20 23 1440 $G 4 3 1 || exit 1; done > $out/pipe_a4.jsonl
cat $out/latency.json
python3 - <<'PY'
import json
for f in ["sealed16.jsonl","pipe.jsonl","pipe_dma.jsonl","pipe_a4.jsonl"]:
    for l in open("gpurun_out/r5c/"+f):
        d=json.loads(l); print(f, {k:d[k] for k in ("seal","groups_per_flush","data_pkt_delay_us_p50","tx_host_ns_per_packet","tx_flush_ms","rx_host_ns_per_packet","rx_flush_ms","all_threads_tx_plus_rx_GiBps")})
PY
