#!/bin/bash
# Round 5: kfec_kernels.hip compiled with LLVM's other scheduler strategies (max-ilp, max-memory-clause,
# iterative-minreg) against the default: 10:3 random-erasure decode, 20:3 headline, 200:55, interleaved.
set -o pipefail
out=gpurun_out/r5x; mkdir -p $out; V=kcptube_amd/variants
L="kcptube_amd/libkfec.so $V/libkfec_k_maxilp.so $V/libkfec_k_maxmemoryclause.so $V/libkfec_k_iterativeminreg.so"
AB_ERASE=random timeout -k 10 300 python tools/ab.py 3 $L -- 10 13 1400 1048576 > $out/ab_103.txt || exit 1
cat $out/ab_103.txt
timeout -k 10 300 python tools/ab.py 2 $L -- 20 23 1440 1048576 > $out/ab_203.txt || exit 1
cat $out/ab_203.txt
AB_ITERS=2 timeout -k 10 400 python tools/ab.py 1 $L -- 200 255 1440 262144 > $out/ab_20055.txt || exit 1
cat $out/ab_20055.txt
