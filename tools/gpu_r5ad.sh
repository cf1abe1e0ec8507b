#!/bin/bash
# Round 5: encode burst loop in word-major MAC order (mb3) against shard-major (shipped): 20:3, 8:4, 10:3.
set -o pipefail
out=gpurun_out/r5ad; mkdir -p $out; V=kcptube_amd/variants
L="kcptube_amd/libkfec.so $V/libkfec_mb3.so"
timeout -k 10 300 python tools/ab.py 3 $L -- 20 23 1440 1048576 > $out/ab_203.txt || exit 1
timeout -k 10 300 python tools/ab.py 2 $L -- 8 12 1440 1048576 > $out/ab_84.txt || exit 1
AB_ERASE=random timeout -k 10 300 python tools/ab.py 2 $L -- 10 13 1400 1048576 > $out/ab_103.txt || exit 1
for f in 203 84 103; do echo "== $f"; cut -c1-110 $out/ab_$f.txt; done
