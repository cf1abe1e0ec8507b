#!/bin/bash
# Round 5: XCD spans (KFEC_XCD_ORDER = S: each XCD takes runs of S adjacent chunks) S = 2, 4, 16 against the
# shipped order, interleaved: 20:3, 10:3 random, 8:4 (parity tests of S = 4 first).
set -o pipefail
out=gpurun_out/r5aj; mkdir -p $out; V=kcptube_amd/variants
KFEC_LIB=$V/libkfec_xcd4.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $out/t1.log 2>&1 || { tail -40 $out/t1.log; exit 1; }
tail -1 $out/t1.log
L="kcptube_amd/libkfec.so $V/libkfec_xcd2.so $V/libkfec_xcd4.so $V/libkfec_xcd16.so"
timeout -k 10 400 python tools/ab.py 3 $L -- 20 23 1440 1048576 > $out/ab_203.txt || exit 1
AB_ERASE=random timeout -k 10 400 python tools/ab.py 3 $L -- 10 13 1400 1048576 > $out/ab_103.txt || exit 1
timeout -k 10 400 python tools/ab.py 2 $L -- 8 12 1440 1048576 > $out/ab_84.txt || exit 1
for f in 203 103 84; do echo "== $f"; cut -c1-150 $out/ab_$f.txt; done
