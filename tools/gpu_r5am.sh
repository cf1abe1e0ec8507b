#!/bin/bash
# Round 5: aes_ocb with four replicated tables (KFEC_OCB_T4=1, variants/libkfec_ocbt4.so): its AEAD parity tests,
# then the bench_aead line (verified) of the shipped build and the variant, interleaved three times.
set -o pipefail
out=gpurun_out/r5am; mkdir -p $out; V=kcptube_amd/variants
KFEC_LIB=$V/libkfec_ocbt4.so timeout -k 10 600 python -u -m pytest tests/test_gpu_aead.py -x -q --timeout 300 --timeout-method thread > $out/t1.log 2>&1 || { tail -40 $out/t1.log; exit 1; }
tail -1 $out/t1.log
for round in 1 2 3; do
for v in base ocbt4; do
  lib=""; [ "$v" != base ] && lib=$V/libkfec_$v.so
  KFEC_LIB=$lib timeout -k 10 300 python -u tools/bench_aead.py --steps 5 > $out/bench_${v}_$round.json 2>$out/bench_$v.err || { tail $out/bench_$v.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$out/bench_${v}_$round.json')); print('$round %-8s' % '$v', ' '.join('%s %.3f/%.3f' % (m, d[m]['seal_ms'], d[m]['open_ms']) for m in ('chacha20','aes_gcm','aes_ocb') if m in d), 'ok' if d['verified'] else 'WRONG')"
done
done
