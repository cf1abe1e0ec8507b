#!/bin/bash
# (r5ao: the lane-0 release form of the count, after r5an measured a per-thread seq_cst system fence)
# Round 5: the small sealed flush / opener flush waiting for the seal kernel's own completion count
# (KFEC_QUEUE_SEAL_COUNT=1, default) against the stream synchronisation (=0): queue / pipeline / frame GPU tests,
# then the sealed deferred delay (checksum16) at 1 / 4 / 16 groups per flush, interleaved twice.
set -o pipefail
out=gpurun_out/r5ao; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_frame.py tests/test_gpu_pipeline.py tests/test_gpu_queue_paths.py -x -q --timeout 120 --timeout-method thread > $out/gtest.log 2>&1 || { tail -40 $out/gtest.log; exit 1; }
tail -1 $out/gtest.log
for rep in 1 2; do for c in 1 0; do
  for g in 1 4 16; do
    KFEC_QUEUE_SEAL_COUNT=$c KFEC_QUEUE_TRACE=1 PB_SEAL=none timeout -k 10 120 ./tools/pipeline_bench 20 23 1440 $g 33 3 1 > $out/s_g${g}_c${c}_$rep.json 2> $out/s_g${g}_c${c}_$rep.err || exit 1
  done
done; done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r5ao/s_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    keys = [k for k in d if "open" in k or "flush" in k]
    print(f.split("/")[-1], "p50", d["data_pkt_delay_us_p50"], "p99", d["data_pkt_delay_us_p99"], {k: d[k] for k in keys[:6]}, open(f.replace(".json", ".err")).read().strip()[-160:].replace("\n", " | "))
PY
