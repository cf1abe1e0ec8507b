#!/bin/bash
# Round 5: flush waits by polling the stream (KFEC_QUEUE_SPIN=1) vs hipStreamSynchronize (0), interleaved twice:
# sealed deferred delay (1 / 4 / 16 groups per flush) and the queues' launch-path flush latency.
set -o pipefail
out=gpurun_out/r5o; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_queue_paths.py tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread > $out/gtest.log 2>&1 || { tail -40 $out/gtest.log; exit 1; }
tail -1 $out/gtest.log
for rep in 1 2; do for sp in 1 0; do
  for mode in none chacha20; do for g in 1 4 16; do
    KFEC_QUEUE_SPIN=$sp KFEC_QUEUE_TRACE=1 PB_SEAL=$mode timeout -k 10 120 ./tools/pipeline_bench 20 23 1440 $g 33 3 1 > $out/s_${mode}_g${g}_sp${sp}_$rep.json 2> $out/s_${mode}_g${g}_sp${sp}_$rep.err || exit 1
  done; done
  KFEC_QUEUE_SPIN=$sp KFEC_QUEUE_WORKER_MAX=0 timeout -k 10 90 ./tools/latency_bench > $out/latq_sp${sp}_$rep.json 2>&1 || exit 1
done; done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r5o/s_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], d["data_pkt_delay_us_p50"], d["data_pkt_delay_us_p99"], "rx_open", d["rx_open_ms"], open(f.replace(".json", ".err")).read().strip()[-100:])
for f in sorted(glob.glob("gpurun_out/r5o/latq_*.json")):
    d = json.load(open(f)); print(f.split("/")[-1], {k: round(v, 1) for k, v in d.items() if "flush" in k})
PY
echo done
