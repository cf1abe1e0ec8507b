#!/bin/bash
# 200:55 coefficient-form decode: LDS per workgroup for the per-chunk tables (l32 shipped, l48, l64 = fewer
# chunks, fewer barriers), parity tests on l64, interleaved timing at 64k groups.
set -o pipefail
V=kcptube_amd/variants; out=gpurun_out/ab_declds; mkdir -p $out
KFEC_LIB=$V/libkfec_l64.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $out/t_l64.log 2>&1 || { tail -30 $out/t_l64.log; exit 1; }
tail -1 $out/t_l64.log
timeout -k 10 600 python tools/ab.py 2 $V/libkfec_l32.so $V/libkfec_l48.so $V/libkfec_l64.so -- 200 255 1440 65536 > $out/ab.txt 2>&1 || { cat $out/ab.txt; exit 1; }
cat $out/ab.txt
