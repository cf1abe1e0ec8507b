#!/bin/bash
# Round 5: decode_prep_lagrange with one wave per group (KFEC_PREP_WAVE=1: four groups per workgroup, no workgroup
# barrier in the group loop; base = 4 waves/SIMD bound, prepw8 = 8) against the workgroup per group (prepwg),
# parity first, then 200:55 and an R = 20 shape, interleaved; kernel times from rocprofv3.
set -o pipefail
out=gpurun_out/r5u; mkdir -p $out; V=kcptube_amd/variants
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $out/t1.log 2>&1 || { tail -40 $out/t1.log; exit 1; }
tail -1 $out/t1.log
KFEC_LIB=$V/libkfec_prepw8.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "batch_vs_oracle" > $out/t2.log 2>&1 || { tail -40 $out/t2.log; exit 1; }
tail -1 $out/t2.log
AB_ITERS=4 timeout -k 10 600 python tools/ab.py 2 kcptube_amd/libkfec.so $V/libkfec_prepw8.so $V/libkfec_prepwg.so -- 200 255 1440 262144 > $out/ab_20055.txt || exit 1
cat $out/ab_20055.txt
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for v in base prepw8 prepwg; do
  lib=""; [ "$v" != base ] && lib=$V/libkfec_$v.so
  KFEC_LIB=$lib AB_ITERS=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt_$v -o kt -- python3 tools/ab_one.py 200 255 1440 262144 > $out/kt_$v.log 2>&1 || exit 1
  grep -h lagrange $out/kt_$v/kt_kernel_stats.csv | cut -d, -f1-4
done
echo done
