#!/bin/bash
# Round 5: sealed checksum flushes emitting their data packets from the host's staged copy
# (KFEC_QUEUE_HOST_DATA=1, shipped) against the sealed rows (0): queue GPU tests, then the deferred delay at
# 4 / 16 groups per flush, interleaved twice; then the syndrome-decode burst / occupancy A/B (gpu_r5aa.sh).
set -o pipefail
out=gpurun_out/r5ab; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_queue_paths.py tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread > $out/gtest.log 2>&1 || { tail -40 $out/gtest.log; exit 1; }
tail -1 $out/gtest.log
for rep in 1 2; do for hd in 1 0; do for g in 1 4 16; do
  KFEC_QUEUE_HOST_DATA=$hd KFEC_QUEUE_TRACE=1 PB_SEAL=none timeout -k 10 120 ./tools/pipeline_bench 20 23 1440 $g 33 3 1 > $out/s_g${g}_hd${hd}_$rep.json 2> $out/s_g${g}_hd${hd}_$rep.err || exit 1
done; done; done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r5ab/s_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], d["data_pkt_delay_us_p50"], d["data_pkt_delay_us_p99"], open(f.replace(".json", ".err")).read().strip()[-110:])
PY
bash tools/gpu_r5aa.sh
