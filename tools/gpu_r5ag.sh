#!/bin/bash
# Round 5: seal / open table staging by 16-byte loads all issued first (KFEC_SEAL_STAGE4=1, shipped) against the
# dword loop (stage1): seal GPU tests, the sealed deferred delay at 1 / 4 / 16 groups per flush (pipeline_bench
# links kcptube_amd/libkfec.so: the variant is copied over it in this box's copy of the tree for its runs), and
# the batched seal / open throughput (bench_seal.py, KFEC_LIB), interleaved twice.
set -o pipefail
out=gpurun_out/r5ag; mkdir -p $out; V=kcptube_amd/variants
timeout -k 10 600 python -u -m pytest tests/test_gpu_frame.py tests/test_gpu_pipeline.py tests/test_gpu_queue_paths.py -x -q --timeout 120 --timeout-method thread > $out/gtest.log 2>&1 || { tail -40 $out/gtest.log; exit 1; }
tail -1 $out/gtest.log
cp kcptube_amd/libkfec.so $out/lib_ship.so
for rep in 1 2; do for v in ship stage1; do
  if [ $v = ship ]; then cp $out/lib_ship.so kcptube_amd/libkfec.so; else cp $V/libkfec_stage1.so kcptube_amd/libkfec.so; fi
  for g in 1 4 16; do
    KFEC_QUEUE_TRACE=1 PB_SEAL=none timeout -k 10 120 ./tools/pipeline_bench 20 23 1440 $g 33 3 1 > $out/s_g${g}_${v}_$rep.json 2> $out/s_g${g}_${v}_$rep.err || exit 1
  done
  timeout -k 10 200 python tools/bench_seal.py > $out/seal_${v}_$rep.json 2>/dev/null || exit 1
done; done
cp $out/lib_ship.so kcptube_amd/libkfec.so
python3 - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r5ag/s_*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], d["data_pkt_delay_us_p50"], d["data_pkt_delay_us_p99"], open(f.replace(".json", ".err")).read().strip()[-100:])
for f in sorted(glob.glob("gpurun_out/r5ag/seal_*.json")):
    print(f.split("/")[-1], open(f).read().strip()[:300])
PY
