#!/bin/bash
# Round 5: the encode burst loop (KFEC_MAC_BURST=2) at other pipeline depths (KFEC_MAC_PD 5 / 3 / 2; shipped 4):
# 20:3, 10:3 and 8:4 encode, interleaved.
set -o pipefail
out=gpurun_out/r5ac; mkdir -p $out; V=kcptube_amd/variants
L="kcptube_amd/libkfec.so $V/libkfec_mpd5.so $V/libkfec_mpd3.so $V/libkfec_mpd2.so"
timeout -k 10 300 python tools/ab.py 3 $L -- 20 23 1440 1048576 > $out/ab_203.txt || exit 1
AB_ERASE=random timeout -k 10 300 python tools/ab.py 2 $L -- 10 13 1400 1048576 > $out/ab_103.txt || exit 1
timeout -k 10 300 python tools/ab.py 2 $L -- 8 12 1440 1048576 > $out/ab_84.txt || exit 1
for f in 203 103 84; do echo "== $f"; cut -c1-110 $out/ab_$f.txt; done
