# round 4: compact syndrome records (KFEC_SYN_REC_COMPACT: 40 + 8 RT bytes, 64 at R = 3) vs 112-byte records
# (rc0): parity through every decode user, prep kernel time under rocprofv3, A/B 10:3 random, 20:3, 20:3 1% loss
set -o pipefail
cd $GRAFT_REPO_ROOT
V=kcptube_amd/variants; O=gpurun_out/r4ab; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_frame.py tests/test_gpu_pipeline.py tests/test_gpu_worker.py -x -q --timeout 200 --timeout-method thread > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for v in rc0 shipped; do
  lib=$V/libkfec_$v.so; [ $v = shipped ] && lib=kcptube_amd/libkfec.so
  AB_ERASE=iid:10000 KFEC_LIB=$PWD/$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$v -o kt -- python3 tools/ab_one.py 20 23 1440 1048576 > $O/prof_$v.log 2>&1 || { tail $O/prof_$v.log; exit 1; }
done
L="$V/libkfec_rc0.so kcptube_amd/libkfec.so"
AB_ERASE=random timeout -k 10 300 python tools/ab.py 3 $L -- 10 13 1400 1048576 > $O/ab_103.txt 2>&1 || { cat $O/ab_103.txt; exit 1; }
cat $O/ab_103.txt
AB_ERASE=iid:10000 timeout -k 10 300 python tools/ab.py 3 $L -- 20 23 1440 1048576 > $O/ab_203loss1.txt 2>&1 || { cat $O/ab_203loss1.txt; exit 1; }
cat $O/ab_203loss1.txt
timeout -k 10 300 python tools/ab.py 2 $L -- 20 23 1440 1048576 > $O/ab_203.txt 2>&1 || { cat $O/ab_203.txt; exit 1; }
cat $O/ab_203.txt
