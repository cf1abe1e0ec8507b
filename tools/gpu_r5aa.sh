#!/bin/bash
# Round 5: the dense syndrome decode with its shard loads as one burst per PD shards (synb) and/or capped at
# 3 / 2 waves per SIMD by LDS (occ3 / occ2), against the shipped build: 20:3 and 10:3 random, interleaved.
set -o pipefail
out=gpurun_out/r5aa; mkdir -p $out; V=kcptube_amd/variants
L="kcptube_amd/libkfec.so $V/libkfec_synb.so $V/libkfec_synb_occ3.so $V/libkfec_syn_occ3.so $V/libkfec_synb_occ2.so"
timeout -k 10 400 python tools/ab.py 3 $L -- 20 23 1440 1048576 > $out/ab_203.txt || exit 1
AB_ERASE=random timeout -k 10 400 python tools/ab.py 3 $L -- 10 13 1400 1048576 > $out/ab_103.txt || exit 1
for f in 203 103; do echo "== $f"; cut -c1-140 $out/ab_$f.txt; done
