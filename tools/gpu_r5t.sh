#!/bin/bash
# Round 5: the R > 8 encode tiles (MT = 8) held to 4 waves per SIMD (KFEC_MINW_ENC8=4: 128 VGPRs, 8 spilled)
# against the default (135 VGPRs, 3 waves), interleaved at 200:55.
set -o pipefail
out=gpurun_out/r5t; mkdir -p $out; V=kcptube_amd/variants
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $out/t1.log 2>&1 || { tail -40 $out/t1.log; exit 1; }
tail -1 $out/t1.log
KFEC_LIB=$V/libkfec_enc8w4.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $out/t2.log 2>&1 || { tail -40 $out/t2.log; exit 1; }
tail -1 $out/t2.log
AB_ITERS=4 timeout -k 10 600 python tools/ab.py 3 kcptube_amd/libkfec.so $V/libkfec_enc8w4.so -- 200 255 1440 262144 > $out/ab_20055.txt || exit 1
cat $out/ab_20055.txt
echo done
