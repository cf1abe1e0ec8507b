# round 4: decode_prep_lagrange capped at 64 VGPRs (KFEC_PREP_MINW 8, 12 spills) vs uncapped: prep kernel time
set -o pipefail
cd $GRAFT_REPO_ROOT
V=kcptube_amd/variants; O=gpurun_out/r4x; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for v in shipped pminw8 shipped2; do
  lib=$V/libkfec_$v.so; [ $v != pminw8 ] && lib=kcptube_amd/libkfec.so
  KFEC_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o kt -- python3 tools/ab_one.py 200 255 1440 262144 > $O/prof_$v.log 2>&1 || { tail $O/prof_$v.log; exit 1; }
done
