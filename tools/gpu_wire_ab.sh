#!/bin/bash
# wire-layer A/B: the frame / pipeline GPU tests of the shipped build, then tools/bench_wire.py for the shipped
# build and each kcptube_amd/variants/libkfec_frame_*.so, interleaved twice (kernel ms per wire kernel).
set -o pipefail
out=gpurun_out/wire_ab; mkdir -p $out
[ -n "$NOTEST" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_frame.py tests/test_gpu_pipeline.py -x -q --timeout 300 --timeout-method thread > $out/gtest.log 2>&1 || { tail -40 $out/gtest.log; exit 1; }
[ -n "$NOTEST" ] || tail -1 $out/gtest.log
for round in 1 2; do
for v in base $(cd kcptube_amd/variants && ls libkfec_frame_*.so 2>/dev/null | sed 's/libkfec_//; s/\.so//'); do
  lib=""; [ "$v" != base ] && lib=kcptube_amd/variants/libkfec_$v.so
  KFEC_LIB=$lib timeout -k 10 300 python -u tools/bench_wire.py --steps 5 > $out/bench_$v.json 2>$out/bench_$v.err || { tail $out/bench_$v.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$out/bench_$v.json')); k=d['kernels']
print('$round %-14s' % '$v', ' '.join('%s %.3f' % (n, t['ms']) for n, t in k.items()), 'send %.3f recv %.3f' % (d['send_ms'], d['recv_ms']))"
done
done
echo ab-done
