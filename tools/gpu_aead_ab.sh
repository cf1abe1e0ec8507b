#!/bin/bash
# AEAD A/B: GPU tests of the shipped build, then the shipped build against the variants in
# kcptube_amd/variants/libkfec_aead_*.so, interleaved twice.
set -o pipefail
out=gpurun_out/aead_ab; mkdir -p $out
[ -n "$NOTEST" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_aead.py -x -q --timeout 300 --timeout-method thread > $out/gtest.log 2>&1 || { tail -40 $out/gtest.log; exit 1; }
[ -n "$NOTEST" ] || tail -1 $out/gtest.log
for round in 1 2; do
for v in base $(cd kcptube_amd/variants && ls libkfec_aead_*.so | sed 's/libkfec_//; s/\.so//'); do
  lib=""; [ "$v" != base ] && lib=kcptube_amd/variants/libkfec_$v.so
  KFEC_LIB=$lib timeout -k 10 300 python -u tools/bench_aead.py --steps 5 --no-verify > $out/bench_$v.json 2>$out/bench_$v.err || { tail $out/bench_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$out/bench_$v.json')); print('$round %-16s' % '$v', ' '.join('%s %.3f/%.3f' % (m, d[m]['seal_ms'], d[m]['open_ms']) for m in ('chacha20','xchacha20','aes_gcm','aes_ocb') if m in d), 'ok' if d['verified'] else 'WRONG')"
done
done
echo ab-done
