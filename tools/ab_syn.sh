#!/bin/bash
# A/B of two syndrome-decode builds (kcptube_amd/variants/libkfec_{A,B}.so): parity tests on B, then
# interleaved timing at 20:3 (3 data shards lost) and 10:3 (1-3 random of 13).  Usage: tools/ab_syn.sh A B
set -o pipefail
A=${1:-wct0}; B=${2:-wct1}; V=kcptube_amd/variants
mkdir -p gpurun_out/ab_syn
KFEC_LIB=$V/libkfec_$B.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ab_syn/t.log 2>&1 || { tail -40 gpurun_out/ab_syn/t.log; exit 1; }
tail -1 gpurun_out/ab_syn/t.log
timeout -k 10 300 python tools/ab.py 3 $V/libkfec_$A.so $V/libkfec_$B.so -- 20 23 1440 1048576 || exit 1
AB_ERASE=random timeout -k 10 300 python tools/ab.py 3 $V/libkfec_$A.so $V/libkfec_$B.so -- 10 13 1400 1048576 || exit 1
