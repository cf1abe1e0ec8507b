#!/bin/bash
# Round 5: counted small sealed flushes with system-scope output stores and no L2 write-back (r5aq) --
# KFEC_QUEUE_SEAL_COUNT=1 against 0 at 1 / 4 / 16 groups per flush, interleaved twice; then the batched seal / open
# throughput of this build against HEAD's (variants/libkfec_head.so: no sys branch in the kernels).
set -o pipefail
out=gpurun_out/r5aq; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_frame.py tests/test_gpu_pipeline.py tests/test_gpu_queue_paths.py -x -q --timeout 120 --timeout-method thread > $out/gtest.log 2>&1 || { tail -40 $out/gtest.log; exit 1; }
tail -1 $out/gtest.log
for rep in 1 2; do for c in 1 0; do
  for g in 1 4 16; do
    KFEC_QUEUE_SEAL_COUNT=$c KFEC_QUEUE_TRACE=1 PB_SEAL=none timeout -k 10 120 ./tools/pipeline_bench 20 23 1440 $g 33 3 1 > $out/s_g${g}_c${c}_$rep.json 2> $out/s_g${g}_c${c}_$rep.err || exit 1
  done
done; done
for rep in 1 2; do
  timeout -k 10 200 python tools/bench_seal.py > $out/seal_new_$rep.json 2>/dev/null || exit 1
  KFEC_LIB=kcptube_amd/variants/libkfec_head.so timeout -k 10 200 python tools/bench_seal.py > $out/seal_head_$rep.json 2>/dev/null || exit 1
done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r5aq/s_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], "p50", d["data_pkt_delay_us_p50"], "p99", d["data_pkt_delay_us_p99"], "rx_open_ms", d.get("rx_open_ms"), open(f.replace(".json", ".err")).read().strip()[-80:].replace("\n", " | "))
for f in sorted(glob.glob("gpurun_out/r5aq/seal_*.json")):
    print(f.split("/")[-1], open(f).read().strip()[:400])
PY
