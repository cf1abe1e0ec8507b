# round 4: compact syndrome kernel (listed groups in the dense item order) -- parity, A/B vs the previous library
set -o pipefail
cd $GRAFT_REPO_ROOT
V=kcptube_amd/variants; O=gpurun_out/r4j; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_frame.py -x -q --timeout 200 --timeout-method thread > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
AB_ERASE=random timeout -k 10 300 python tools/ab.py 3 $V/libkfec_base.so kcptube_amd/libkfec.so -- 10 13 1400 1048576 > $O/ab_103.txt 2>&1 || { cat $O/ab_103.txt; exit 1; }
cat $O/ab_103.txt
timeout -k 10 300 python tools/ab.py 2 $V/libkfec_base.so kcptube_amd/libkfec.so -- 20 23 1440 1048576 > $O/ab_203.txt 2>&1 || { cat $O/ab_203.txt; exit 1; }
cat $O/ab_203.txt
AB_ERASE=iid:10000 timeout -k 10 300 python tools/ab.py 2 $V/libkfec_base.so kcptube_amd/libkfec.so -- 20 23 1440 1048576 > $O/ab_203loss1.txt 2>&1 || { cat $O/ab_203loss1.txt; exit 1; }
cat $O/ab_203loss1.txt
