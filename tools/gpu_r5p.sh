#!/bin/bash
# Round 5: the syndrome decode's arithmetic-free bound -- the same kernel with every GF multiply-accumulate
# replaced by a plain XOR (KFEC_SYN_XORONLY, same loads / stores / tables; wrong results, timing only), against the
# shipped kernel, interleaved: 10:3 with random 1-3 erasures of 13, and 20:3 with 3 data shards lost.
set -o pipefail
out=gpurun_out/r5p; mkdir -p $out; V=kcptube_amd/variants
AB_ERASE=random timeout -k 10 300 python tools/ab.py 3 kcptube_amd/libkfec.so $V/libkfec_xoronly.so -- 10 13 1400 1048576 > $out/ab_103.txt || exit 1
cat $out/ab_103.txt
timeout -k 10 300 python tools/ab.py 2 kcptube_amd/libkfec.so $V/libkfec_xoronly.so -- 20 23 1440 1048576 > $out/ab_203.txt || exit 1
cat $out/ab_203.txt
echo done
