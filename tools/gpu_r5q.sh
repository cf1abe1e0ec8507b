#!/bin/bash
# Round 5: the small sealed flush with its seal launch queued behind a stream gate before the worker request
# (KFEC_QUEUE_GATE=1, default; KFEC_QUEUE_SEAL_SPLIT=1: data packets' seal ahead of the gate) against the seal
# launch after the worker (KFEC_QUEUE_GATE=0): queue GPU tests first, then sealed delay at 1 / 4 / 16 groups.
set -o pipefail
out=gpurun_out/r5q; mkdir -p $out
timeout -k 10 900 python -u -m pytest tests/test_gpu_queue_paths.py tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread > $out/gtest.log 2>&1 || { tail -40 $out/gtest.log; exit 1; }
tail -1 $out/gtest.log
KFEC_QUEUE_SEAL_SPLIT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_queue_paths.py -x -q --timeout 120 --timeout-method thread -k sealed > $out/gtest_split.log 2>&1 || { tail -40 $out/gtest_split.log; exit 1; }
tail -1 $out/gtest_split.log
for rep in 1 2; do for v in "1 0" "1 1" "0 0"; do set -- $v
  for mode in none chacha20 aes_gcm; do for g in 1 4 16; do
    KFEC_QUEUE_GATE=$1 KFEC_QUEUE_SEAL_SPLIT=$2 KFEC_QUEUE_TRACE=1 PB_SEAL=$mode timeout -k 10 120 ./tools/pipeline_bench 20 23 1440 $g 33 3 1 > $out/s_${mode}_g${g}_gate$1_split$2_$rep.json 2> $out/s_${mode}_g${g}_gate$1_split$2_$rep.err || exit 1
  done; done
done; done
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r5q/s_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], d["data_pkt_delay_us_p50"], d["data_pkt_delay_us_p99"], open(f.replace(".json", ".err")).read().strip()[-105:])
PY
echo done
