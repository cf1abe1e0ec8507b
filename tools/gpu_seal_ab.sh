#!/bin/bash
# seal/open A/B: the GPU seal tests of the shipped build, then bench_seal.py for the shipped build and each
# kcptube_amd/variants/libkfec_seal_*.so, interleaved twice.
set -o pipefail
out=gpurun_out/seal_ab; mkdir -p $out
[ -n "$NOTEST" ] || timeout -k 10 600 python -u -m pytest tests/test_gpu_frame.py -x -q --timeout 300 --timeout-method thread -k "seal or open" > $out/gtest.log 2>&1 || { tail -40 $out/gtest.log; exit 1; }
[ -n "$NOTEST" ] || tail -1 $out/gtest.log
for round in 1 2; do
for v in base $(cd kcptube_amd/variants && ls libkfec_seal_*.so | sed 's/libkfec_//; s/\.so//'); do
  lib=""; [ "$v" != base ] && lib=kcptube_amd/variants/libkfec_$v.so
  # exit 3 = ran but verification failed: expected for the ablation builds (*_ab_*), which skip work
  KFEC_LIB=$lib timeout -k 10 300 python -u tools/bench_seal.py --steps 5 > $out/bench_$v.json 2>$out/bench_$v.err; rc=$?
  [ $rc = 0 ] || { [ $rc = 3 ] && [[ $v == *_ab_* ]]; } || { tail $out/bench_$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$out/bench_$v.json')); print('$round %-12s' % '$v', ' '.join('%s %.3f/%.3f' % (m, d[m]['seal_ms'], d[m]['open_ms']) for m in ('none','plain_xor','none_in_place')), 'ok' if d['verified'] else 'WRONG')"
done
done
echo ab-done
