#!/bin/bash
# Round 5: B = 1400 rows at a 1408-byte pitch (aligned rows, the 24-byte tail granule kept) against B = 1400 and
# B = 1408 back to back: does the 10:3 / 20:3 gap come from row alignment or from the tail granule?
set -o pipefail
out=gpurun_out/r5ah; mkdir -p $out
for rep in 1 2; do for cfg in "1400 0" "1400 1408" "1408 0" "1440 0" "1440 1472" "1440 1536"; do set -- $cfg
  AB_PITCH=$2 AB_ERASE=random timeout -k 10 200 python tools/ab.py 1 kcptube_amd/libkfec.so -- 10 13 $1 1048576 > $out/r_${1}_${2}_$rep.txt || exit 1
  AB_PITCH=$2 timeout -k 10 200 python tools/ab.py 1 kcptube_amd/libkfec.so -- 20 23 $1 1048576 > $out/d_${1}_${2}_$rep.txt || exit 1
  echo "B=$1 pitch=$2 10:3r $(cut -c30-200 $out/r_${1}_${2}_$rep.txt) | 20:3 $(cut -c30-200 $out/d_${1}_${2}_$rep.txt)"
done; done
