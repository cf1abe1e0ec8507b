#!/bin/bash
# Round 5 (r5aw): the encode MAC's granules in flight (KFEC_MAC_PD 3 / 6 against the shipped 4) under the XCD spans:
# 20:3, 10:3 random, 8:4, interleaved.
set -o pipefail
out=gpurun_out/r5aw; mkdir -p $out; V=kcptube_amd/variants
L="kcptube_amd/libkfec.so $V/libkfec_mpd3.so $V/libkfec_mpd6.so"
timeout -k 10 300 python tools/ab.py 3 $L -- 20 23 1440 1048576 > $out/ab_203.txt || exit 1
AB_ERASE=random timeout -k 10 300 python tools/ab.py 2 $L -- 10 13 1400 1048576 > $out/ab_103.txt || exit 1
timeout -k 10 300 python tools/ab.py 2 $L -- 8 12 1440 1048576 > $out/ab_84.txt || exit 1
python3 tools/ab_summary.py $out/ab_*.txt
