#!/bin/bash
# Round 5: the 20:3 encode MAC at fewer waves per SIMD (LDS-capped: occ3 / occ4), a deeper load pipeline (pd6),
# and the iterative-minreg schedule (133 VGPRs, 3 waves) against the shipped build, interleaved.
set -o pipefail
out=gpurun_out/r5y; mkdir -p $out; V=kcptube_amd/variants
L="kcptube_amd/libkfec.so $V/libkfec_burst2.so $V/libkfec_burst2_w4.so $V/libkfec_k_minreg.so"
timeout -k 10 400 python tools/ab.py 3 $L -- 20 23 1440 1048576 > $out/ab_203.txt || exit 1
cat $out/ab_203.txt
AB_ERASE=random timeout -k 10 300 python tools/ab.py 2 $L -- 10 13 1400 1048576 > $out/ab_103.txt || exit 1
cat $out/ab_103.txt
