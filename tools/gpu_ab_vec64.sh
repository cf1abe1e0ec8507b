#!/bin/bash
# 10:3 syndrome decode with 64-byte granules (two columns per lane, v64p2 / v64p3 = 2 / 3 granules in flight)
# against the 32-byte shape (v32): parity tests on each 64-byte build, then interleaved timing, 10:3 random 1-3
# of 13 and 5:2 random.
set -o pipefail
V=kcptube_amd/variants; out=gpurun_out/ab_vec64; mkdir -p $out
for b in v64p2 v64p3; do
  KFEC_LIB=$V/libkfec_$b.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $out/t_$b.log 2>&1 || { tail -30 $out/t_$b.log; exit 1; }
  echo "$b: $(tail -1 $out/t_$b.log)"
done
AB_ERASE=random timeout -k 10 400 python tools/ab.py 3 $V/libkfec_v32.so $V/libkfec_v64p2.so $V/libkfec_v64p3.so -- 10 13 1400 1048576 > $out/ab_103.txt 2>&1 || { cat $out/ab_103.txt; exit 1; }
cat $out/ab_103.txt
