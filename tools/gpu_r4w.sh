# round 4: decode_prep_lagrange: prep0 = two loops, prep1 = one fused pass (KFEC_PREP_FUSED), prep2 = + coefficients from stored column points without a modulo (KFEC_PREP_COEF2), shipped = + next group's present bits one group ahead (KFEC_PREP_PREFETCH)
# parity (the R > 8 oracle cases), prep kernel time under rocprofv3 per build, interleaved 200:55 A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
V=kcptube_amd/variants; O=gpurun_out/r4w; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for v in prep0 prep1 prep2 shipped; do
  lib=$V/libkfec_$v.so; [ $v = shipped ] && lib=kcptube_amd/libkfec.so
  KFEC_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o kt -- python3 tools/ab_one.py 200 255 1440 262144 > $O/prof_$v.log 2>&1 || { tail $O/prof_$v.log; exit 1; }
done
L="$V/libkfec_prep0.so $V/libkfec_prep1.so $V/libkfec_prep2.so kcptube_amd/libkfec.so"
timeout -k 10 500 python tools/ab.py 2 $L -- 200 255 1440 262144 > $O/ab_20055.txt 2>&1 || { cat $O/ab_20055.txt; exit 1; }
cat $O/ab_20055.txt
