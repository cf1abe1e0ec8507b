#!/bin/bash
# Round 5 (r5as): the completion count for the AEAD modes' small sealed flushes and opener flushes too --
# KFEC_QUEUE_SEAL_COUNT=1 against 0, chacha20 / aes_gcm / aes_ocb at 1 / 2 / 4 groups per flush, interleaved once.
set -o pipefail
out=gpurun_out/r5as; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_aead.py tests/test_gpu_pipeline.py tests/test_gpu_queue_paths.py -x -q --timeout 120 --timeout-method thread > $out/gtest.log 2>&1 || { tail -40 $out/gtest.log; exit 1; }
tail -1 $out/gtest.log
for rep in 1; do for c in 1 0; do for m in chacha20 aes_gcm aes_ocb; do
  for g in 1 2 4; do
    KFEC_QUEUE_SEAL_COUNT=$c KFEC_QUEUE_TRACE=1 PB_SEAL=$m timeout -k 10 120 ./tools/pipeline_bench 20 23 1440 $g 33 3 1 > $out/s_${m}_g${g}_c${c}_$rep.json 2> $out/s_${m}_g${g}_c${c}_$rep.err || exit 1
  done
done; done; done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r5as/s_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], "p50", d["data_pkt_delay_us_p50"], "p99", d["data_pkt_delay_us_p99"], "rx_open_ms", d.get("rx_open_ms"), open(f.replace(".json", ".err")).read().strip().splitlines()[-1].split("us each:")[-1])
PY
