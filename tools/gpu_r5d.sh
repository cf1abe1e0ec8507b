#!/bin/bash
# Round 5: bucketed syndrome decode (parity + A/B), sealed small flush on the queue's own stream,
# BAR-mode vs DMA staging throughput.
set -o pipefail
out=gpurun_out/r5d; mkdir -p $out; V=kcptube_amd/variants
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_frame.py tests/test_gpu_queue_paths.py -x -q --timeout 120 --timeout-method thread > $out/t1.log 2>&1 || { tail -40 $out/t1.log; exit 1; }
tail -2 $out/t1.log
timeout -k 10 300 python tools/ab.py 3 $V/libkfec_bk0.so $V/libkfec_bk1.so -- 20 23 1440 1048576 > $out/ab_203.txt || exit 1
AB_ERASE=random timeout -k 10 300 python tools/ab.py 3 $V/libkfec_bk0.so $V/libkfec_bk1.so -- 10 13 1400 1048576 > $out/ab_103.txt || exit 1
AB_ERASE=iid:10000 timeout -k 10 300 python tools/ab.py 3 $V/libkfec_bk0.so $V/libkfec_bk1.so -- 20 23 1440 1048576 > $out/ab_loss1.txt || exit 1
cat $out/ab_*.txt
for mode in none chacha20 aes_gcm; do PB_SEAL=$mode timeout -k 10 120 ./tools/pipeline_bench 20 23 1440 16 33 3 1 || exit 1; done > $out/sealed16.jsonl
for G in 4096 16384; do timeout -k 10 300 ./tools/pipeline_bench 20 23 1440 $G 8 3 1 || exit 1; KFEC_QUEUE_BAR=0 timeout -k 10 300 ./tools/pipeline_bench 20 23 1440 $G 8 3 1 || exit 1; done > $out/pipe.jsonl
timeout -k 10 120 ./tools/latency_bench > $out/latency.json 2>&1 || { cat $out/latency.json; exit 1; }
python3 - <<'PY'
import json
for f in ["sealed16.jsonl","pipe.jsonl"]:
    for l in open("gpurun_out/r5d/"+f):
        d=json.loads(l); print(f, {k:d[k] for k in ("seal","groups_per_flush","data_pkt_delay_us_p50","data_pkt_delay_us_p99","tx_host_ns_per_packet","tx_flush_ms","rx_host_ns_per_packet","rx_flush_ms","all_threads_tx_plus_rx_GiBps")})
d=json.load(open("gpurun_out/r5d/latency.json")); print({k:round(v,1) for k,v in d.items() if "flush" in k})
PY
