#!/bin/bash
# Round 5 (r5au): XCD spans in the framed encode / decode kernels (KFEC_XCD_FRAME=1, this build) against the plain
# order (variants/libkfec_frame0.so): frame / pipeline GPU tests, then bench_wire.py interleaved twice.
set -o pipefail
out=gpurun_out/r5au; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_frame.py tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread > $out/gtest.log 2>&1 || { tail -40 $out/gtest.log; exit 1; }
tail -1 $out/gtest.log
for rep in 1 2; do
  timeout -k 10 200 python tools/bench_wire.py > $out/wire_span_$rep.json 2>/dev/null || exit 1
  KFEC_LIB=kcptube_amd/variants/libkfec_frame0.so timeout -k 10 200 python tools/bench_wire.py > $out/wire_plain_$rep.json 2>/dev/null || exit 1
done
for f in $out/wire_*.json; do echo "$f $(cut -c1-700 $f)"; done
