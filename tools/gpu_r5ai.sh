#!/bin/bash
# Round 5: XCD-contiguous chunk order for the single-tile MAC and dense syndrome launches (KFEC_XCD_ORDER=1,
# variants/libkfec_xcd.so) against the shipped order: its parity tests, then interleaved A/B over 20:3,
# 10:3 random, 20:3 at 1% loss, 8:4.
set -o pipefail
out=gpurun_out/r5ai; mkdir -p $out; V=kcptube_amd/variants
KFEC_LIB=$V/libkfec_xcd.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $out/t1.log 2>&1 || { tail -40 $out/t1.log; exit 1; }
tail -1 $out/t1.log
L="kcptube_amd/libkfec.so $V/libkfec_xcd.so"
timeout -k 10 300 python tools/ab.py 4 $L -- 20 23 1440 1048576 > $out/ab_203.txt || exit 1
AB_ERASE=random timeout -k 10 300 python tools/ab.py 4 $L -- 10 13 1400 1048576 > $out/ab_103.txt || exit 1
AB_ERASE=iid:10000 timeout -k 10 300 python tools/ab.py 2 $L -- 20 23 1440 1048576 > $out/ab_loss1.txt || exit 1
timeout -k 10 300 python tools/ab.py 2 $L -- 8 12 1440 1048576 > $out/ab_84.txt || exit 1
for f in 203 103 loss1 84; do echo "== $f"; cut -c1-160 $out/ab_$f.txt; done
