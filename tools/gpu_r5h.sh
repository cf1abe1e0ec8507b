#!/bin/bash
# Round 5: sealed small flush with the data packets' seal launched ahead of (and running beside) the worker's
# parity; queue flush latency after the upload-drain fix.
set -o pipefail
out=gpurun_out/r5h; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_queue_paths.py tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread > $out/gtest.log 2>&1 || { tail -40 $out/gtest.log; exit 1; }
tail -1 $out/gtest.log
for mode in none chacha20 aes_gcm; do
  KFEC_QUEUE_TRACE=1 PB_SEAL=$mode timeout -k 10 120 ./tools/pipeline_bench 20 23 1440 16 33 3 1 > $out/sealed_$mode.json 2> $out/sealed_$mode.err || exit 1
done
for i in 1 2; do timeout -k 10 90 ./tools/latency_bench > $out/latency_$i.json 2>&1 || { cat $out/latency_$i.json; exit 1; }; done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r5h/sealed_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], {k: d[k] for k in ("data_pkt_delay_us_p50", "data_pkt_delay_us_p99", "tx_host_ns_per_packet", "tx_flush_ms", "rx_open_ms", "rx_flush_ms")}, open(f.replace(".json", ".err")).read().strip()[-200:])
for f in sorted(glob.glob("gpurun_out/r5h/latency_*.json")):
    d = json.load(open(f))
    print(f.split("/")[-1], {k: round(v, 1) for k, v in d.items() if "flush" in k})
PY
echo done
