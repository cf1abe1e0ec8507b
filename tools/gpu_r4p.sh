# round 4: syndrome decode computes only the parity rows a wave uses (KFEC_SYN_ROWMASK) -- parity on the
# shipped build (mask 1), then A/B: HEAD before the change, mask 0 / 1 / 2
set -o pipefail
cd $GRAFT_REPO_ROOT
V=kcptube_amd/variants; O=gpurun_out/r4p; mkdir -p $O
L="$V/libkfec_base.so $V/libkfec_rm0.so kcptube_amd/libkfec.so $V/libkfec_rm2.so"
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_frame.py -x -q --timeout 200 --timeout-method thread > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
AB_ERASE=random timeout -k 10 300 python tools/ab.py 3 $L -- 10 13 1400 1048576 > $O/ab_103.txt 2>&1 || { cat $O/ab_103.txt; exit 1; }
cat $O/ab_103.txt
AB_ERASE=iid:10000 timeout -k 10 300 python tools/ab.py 2 $L -- 20 23 1440 1048576 > $O/ab_203loss1.txt 2>&1 || { cat $O/ab_203loss1.txt; exit 1; }
cat $O/ab_203loss1.txt
timeout -k 10 300 python tools/ab.py 2 $L -- 20 23 1440 1048576 > $O/ab_203.txt 2>&1 || { cat $O/ab_203.txt; exit 1; }
cat $O/ab_203.txt
