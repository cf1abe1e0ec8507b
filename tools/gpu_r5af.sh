#!/bin/bash
# Round 5: is the 10:3 random decode's gap the B = 1400 tail granule (43 full 32-byte granules + 24 bytes)?
# Same shape at B = 1400, 1408 (44 x 32) and 1440 (45 x 32), random 1-3 erasures of 13, two rounds.
set -o pipefail
out=gpurun_out/r5af; mkdir -p $out
for rep in 1 2; do for B in 1400 1408 1440; do
  AB_ERASE=random timeout -k 10 200 python tools/ab.py 1 kcptube_amd/libkfec.so -- 10 13 $B 1048576 > $out/ab_${B}_$rep.txt || exit 1
  echo "B=$B $(cut -c1-160 $out/ab_${B}_$rep.txt)"
done; done
