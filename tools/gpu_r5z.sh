#!/bin/bash
# Round 5: encode MAC with table / load bursts (KFEC_MAC_BURST=2, shipped) against the interleaved loop (burst0):
# parity tests, then 20:3, 10:3 random, 20:1 (MT 1), 8:4 (MT 4) and 200:55 (unchanged shape), interleaved.
set -o pipefail
out=gpurun_out/r5z; mkdir -p $out; V=kcptube_amd/variants
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_worker.py -x -q --timeout 200 --timeout-method thread > $out/t1.log 2>&1 || { tail -40 $out/t1.log; exit 1; }
tail -1 $out/t1.log
L="kcptube_amd/libkfec.so $V/libkfec_burst0.so"
timeout -k 10 300 python tools/ab.py 3 $L -- 20 23 1440 1048576 > $out/ab_203.txt || exit 1
AB_ERASE=random timeout -k 10 300 python tools/ab.py 3 $L -- 10 13 1400 1048576 > $out/ab_103.txt || exit 1
timeout -k 10 300 python tools/ab.py 2 $L -- 20 21 1440 1048576 > $out/ab_201.txt || exit 1
timeout -k 10 300 python tools/ab.py 2 $L -- 8 12 1440 1048576 > $out/ab_84.txt || exit 1
AB_ITERS=2 timeout -k 10 300 python tools/ab.py 1 $L -- 200 255 1440 262144 > $out/ab_20055.txt || exit 1
for f in 203 103 201 84 20055; do echo "== $f"; cut -c1-140 $out/ab_$f.txt; done
