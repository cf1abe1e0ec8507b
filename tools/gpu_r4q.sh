# round 4: syndrome decode prologue (KFEC_SYN_EARLY) and E-table prefetch (KFEC_SYN_TPRE): parity on the shipped build and on tpre, A/B against HEAD
set -o pipefail
cd $GRAFT_REPO_ROOT
V=kcptube_amd/variants; O=gpurun_out/r4q; mkdir -p $O
L="$V/libkfec_base.so $V/libkfec_early0.so kcptube_amd/libkfec.so $V/libkfec_tpre.so"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_frame.py -x -q --timeout 200 --timeout-method thread > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
KFEC_LIB=$V/libkfec_tpre.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/parity_tpre.log 2>&1 || { tail -30 $O/parity_tpre.log; exit 1; }
tail -1 $O/parity_tpre.log
AB_ERASE=random timeout -k 10 300 python tools/ab.py 3 $L -- 10 13 1400 1048576 > $O/ab_103.txt 2>&1 || { cat $O/ab_103.txt; exit 1; }
cat $O/ab_103.txt
AB_ERASE=iid:10000 timeout -k 10 300 python tools/ab.py 2 $L -- 20 23 1440 1048576 > $O/ab_203loss1.txt 2>&1 || { cat $O/ab_203loss1.txt; exit 1; }
cat $O/ab_203loss1.txt
timeout -k 10 300 python tools/ab.py 2 $L -- 20 23 1440 1048576 > $O/ab_203.txt 2>&1 || { cat $O/ab_203.txt; exit 1; }
cat $O/ab_203.txt
