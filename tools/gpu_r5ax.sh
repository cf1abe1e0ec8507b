#!/bin/bash
# Round 5 (r5ax): sealed deferred data-packet delay on the final build (completion count on), checksum16 / chacha20 /
# aes_gcm at 1 / 2 / 4 / 8 / 16 groups per flush.
set -o pipefail
out=gpurun_out/r5ax; mkdir -p $out
for m in none chacha20 aes_gcm; do for g in 1 2 4 8 16; do
  KFEC_QUEUE_TRACE=1 PB_SEAL=$m timeout -k 10 120 ./tools/pipeline_bench 20 23 1440 $g 33 3 1 > $out/s_${m}_g$g.json 2> $out/s_${m}_g$g.err || exit 1
done; done
python3 - <<'PY'
import json, glob
rows = []
for m in ("none", "chacha20", "aes_gcm"):
    for g in (1, 2, 4, 8, 16):
        f = f"gpurun_out/r5ax/s_{m}_g{g}.json"
        d = json.loads(open(f).read().strip().splitlines()[-1])
        rows.append({"mode": m, "groups_per_flush": g, "p50_us": d["data_pkt_delay_us_p50"], "p99_us": d["data_pkt_delay_us_p99"],
                     "rx_open_ms": d.get("rx_open_ms"), "phases": open(f.replace(".json", ".err")).read().strip().splitlines()[-1]})
json.dump({"what": "sealed deferred data packets, send -> emission delay (tools/pipeline_bench, fec=20:3, kcp_mtu 1440, one host thread), final round-5 build", "rows": rows}, open("gpurun_out/r5ax/sweep.json", "w"), indent=1)
for r in rows: print(r["mode"], r["groups_per_flush"], r["p50_us"], r["p99_us"], r["rx_open_ms"])
PY
