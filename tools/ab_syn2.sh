#!/bin/bash
# A/B of several syndrome-decode builds (kcptube_amd/variants/libkfec_<name>.so): parity tests on the builds
# named in $CHECK, then interleaved timing at 10:3 (1-3 random of 13) and 20:3 (3 data shards lost).
# Usage: CHECK="e1 p12" tools/ab_syn2.sh e0 e1 p6 ...
set -o pipefail
V=kcptube_amd/variants; out=gpurun_out/ab_syn2; mkdir -p $out
for b in $CHECK; do
  KFEC_LIB=$V/libkfec_$b.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $out/t_$b.log 2>&1 || { tail -40 $out/t_$b.log; exit 1; }
  echo "$b: $(tail -1 $out/t_$b.log)"
done
libs=""; for b in "$@"; do libs="$libs $V/libkfec_$b.so"; done
AB_ERASE=random timeout -k 10 400 python tools/ab.py ${ROUNDS:-3} $libs -- 10 13 1400 1048576 || exit 1
timeout -k 10 400 python tools/ab.py ${ROUNDS:-3} $libs -- 20 23 1440 1048576 || exit 1
AB_ERASE=iid:10000 timeout -k 10 400 python tools/ab.py ${ROUNDS:-3} $libs -- 20 23 1440 1048576 || exit 1
