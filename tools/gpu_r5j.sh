#!/bin/bash
# Round 5: sealed deferred data-packet delay against the flush size (1 .. 16 groups per flush), with phase traces.
set -o pipefail
out=gpurun_out/r5j; mkdir -p $out
for mode in none chacha20 aes_gcm; do
  for g in 1 2 4 8 16; do
    f=$(( g >= 8 ? 33 : 65 ))
    KFEC_QUEUE_TRACE=1 PB_SEAL=$mode timeout -k 10 120 ./tools/pipeline_bench 20 23 1440 $g $f 3 1 > $out/sealed_${mode}_g$g.json 2> $out/sealed_${mode}_g$g.err || exit 1
  done
done
python3 - <<'PY'
import json, glob
rows = {}
for f in sorted(glob.glob("gpurun_out/r5j/sealed_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    name = f.split("/")[-1][:-5]
    print(name, {k: d[k] for k in ("data_pkt_delay_us_p50", "data_pkt_delay_us_p90", "data_pkt_delay_us_p99", "tx_host_ns_per_packet", "tx_flush_ms")}, open(f.replace(".json", ".err")).read().strip()[-170:])
PY
echo done
