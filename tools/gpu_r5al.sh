#!/bin/bash
# Round 5: XCD spans S = 16 and 64 against the shipped order, a second box: 20:3, 10:3 random, 20:3 at 1% loss.
set -o pipefail
out=gpurun_out/r5al; mkdir -p $out; V=kcptube_amd/variants
L="kcptube_amd/libkfec.so $V/libkfec_xcd16.so $V/libkfec_xcd64.so"
timeout -k 10 400 python tools/ab.py 4 $L -- 20 23 1440 1048576 > $out/ab_203.txt || exit 1
AB_ERASE=random timeout -k 10 400 python tools/ab.py 3 $L -- 10 13 1400 1048576 > $out/ab_103.txt || exit 1
AB_ERASE=iid:10000 timeout -k 10 400 python tools/ab.py 2 $L -- 20 23 1440 1048576 > $out/ab_loss1.txt || exit 1
