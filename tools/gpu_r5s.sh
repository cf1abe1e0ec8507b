#!/bin/bash
# Round 5: the listed syndrome kernel (one group per wave, only the group's present rows loaded, per-group row
# masks) forced for the dense shapes too (KFEC_SYN_FORCE_LIST) against the dense kernel, interleaved.
set -o pipefail
out=gpurun_out/r5s; mkdir -p $out; V=kcptube_amd/variants
AB_ERASE=random timeout -k 10 300 python tools/ab.py 3 kcptube_amd/libkfec.so $V/libkfec_forcelist.so -- 10 13 1400 1048576 > $out/ab_103.txt || exit 1
cat $out/ab_103.txt
timeout -k 10 300 python tools/ab.py 2 kcptube_amd/libkfec.so $V/libkfec_forcelist.so -- 20 23 1440 1048576 > $out/ab_203.txt || exit 1
cat $out/ab_203.txt
echo done
