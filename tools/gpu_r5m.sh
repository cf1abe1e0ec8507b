#!/bin/bash
# Round 5: emission prefetch (KFEC_QUEUE_PREFETCH) A/B: sealed deferred delay at 4 / 16 groups per flush and the
# small-flush latency, interleaved 1 / 0 twice.
set -o pipefail
out=gpurun_out/r5m2; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_queue_paths.py -x -q --timeout 120 --timeout-method thread > $out/gtest.log 2>&1 || { tail -40 $out/gtest.log; exit 1; }
tail -1 $out/gtest.log
for rep in 1 2; do for pf in 1 0; do
  for mode in none chacha20; do for g in 4 16; do
    KFEC_QUEUE_PREFETCH=$pf KFEC_QUEUE_TRACE=1 PB_SEAL=$mode timeout -k 10 120 ./tools/pipeline_bench 20 23 1440 $g 33 3 1 > $out/s_${mode}_g${g}_pf${pf}_$rep.json 2> $out/s_${mode}_g${g}_pf${pf}_$rep.err || exit 1
  done; done
  KFEC_QUEUE_PREFETCH=$pf timeout -k 10 90 ./tools/latency_bench > $out/lat_pf${pf}_$rep.json 2>&1 || exit 1
done; done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r5m2/s_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], d["data_pkt_delay_us_p50"], d["data_pkt_delay_us_p99"], "rx_open", d["rx_open_ms"], "rx_flush", d["rx_flush_ms"], open(f.replace(".json", ".err")).read().strip()[-110:])
for f in sorted(glob.glob("gpurun_out/r5m2/lat_*.json")):
    d = json.load(open(f)); print(f.split("/")[-1], {k: round(v, 1) for k, v in d.items() if "flush" in k})
PY
echo done
