#!/bin/bash
# Round 5: coherent host outputs for the small sealed / open flushes (A/B), with phase traces.
set -o pipefail
out=gpurun_out/r5g; mkdir -p $out
for c in 1 0; do for mode in none chacha20; do
  KFEC_QUEUE_COHERENT_OUT=$c KFEC_QUEUE_TRACE=1 PB_SEAL=$mode timeout -k 10 120 ./tools/pipeline_bench 20 23 1440 16 33 3 1 > $out/sealed_${mode}_c$c.json 2> $out/sealed_${mode}_c$c.err || exit 1
done; done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r5g/sealed_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], {k: d[k] for k in ("data_pkt_delay_us_p50", "data_pkt_delay_us_p99", "tx_host_ns_per_packet", "tx_flush_ms", "rx_open_ms", "rx_flush_ms")}, open(f.replace(".json", ".err")).read().strip()[-150:])
PY
