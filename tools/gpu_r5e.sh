#!/bin/bash
# Round 5: worker stream priority (sealed small flush), queue initial mode, factored 200:55 decode records.
set -o pipefail
out=gpurun_out/r5e; mkdir -p $out; V=kcptube_amd/variants
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_queue_paths.py tests/test_gpu_pipeline.py -x -q --timeout 200 --timeout-method thread > $out/t1.log 2>&1 || { tail -40 $out/t1.log; exit 1; }
tail -2 $out/t1.log
for mode in none chacha20 aes_gcm; do PB_SEAL=$mode timeout -k 10 120 ./tools/pipeline_bench 20 23 1440 16 33 3 1 || exit 1; done > $out/sealed16.jsonl
timeout -k 10 300 ./tools/pipeline_bench 20 23 1440 16384 8 3 1 > $out/pipe.jsonl || exit 1
KFEC_QUEUE_BAR=0 timeout -k 10 300 ./tools/pipeline_bench 20 23 1440 16384 8 3 1 >> $out/pipe.jsonl || exit 1
timeout -k 10 120 ./tools/latency_bench > $out/latency.json 2>&1 || { cat $out/latency.json; exit 1; }
python3 - <<'PY'
import json
for f in ["sealed16.jsonl","pipe.jsonl"]:
    for l in open("gpurun_out/r5e/"+f):
        d=json.loads(l); print(f, {k:d[k] for k in ("seal","groups_per_flush","data_pkt_delay_us_p50","data_pkt_delay_us_p99","tx_host_ns_per_packet","tx_flush_ms","rx_host_ns_per_packet","rx_flush_ms","all_threads_tx_plus_rx_GiBps")})
d=json.load(open("gpurun_out/r5e/latency.json")); print({k:round(v,1) for k,v in d.items() if "flush" in k})
PY
AB_ITERS=4 timeout -k 10 600 python tools/ab.py 2 $V/libkfec_fac0.so $V/libkfec_fac1.so -- 200 255 1440 262144 > $out/ab_20055.txt || exit 1
cat $out/ab_20055.txt
