#!/bin/bash
# Round 5: syndrome decode start-up -- the record header requested before the list count (scalar) is checked
# (KFEC_SYN_HDR_FIRST) and the first PD data granules requested before the header arrives (KFEC_SYN_SPEC).
# base = both; spec0 = header first only; hdr0 = neither (round 4's order). Interleaved A/B, three shapes.
set -o pipefail
out=gpurun_out/r5l; mkdir -p $out; V=kcptube_amd/variants
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $out/t1.log 2>&1 || { tail -40 $out/t1.log; exit 1; }
tail -1 $out/t1.log
L="kcptube_amd/libkfec.so $V/libkfec_spec0.so $V/libkfec_hdr0.so"
AB_ERASE=random timeout -k 10 300 python tools/ab.py 3 $L -- 10 13 1400 1048576 > $out/ab_103.txt || exit 1
cat $out/ab_103.txt
timeout -k 10 300 python tools/ab.py 2 $L -- 20 23 1440 1048576 > $out/ab_203.txt || exit 1
cat $out/ab_203.txt
AB_ERASE=iid:10000 timeout -k 10 300 python tools/ab.py 2 $L -- 20 23 1440 1048576 > $out/ab_loss1.txt || exit 1
cat $out/ab_loss1.txt
echo done
