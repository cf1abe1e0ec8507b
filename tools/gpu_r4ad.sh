# round 4: dense syndrome kernel with KFEC_SYN_CPW consecutive chunks per workgroup (libkfec = HEAD, one chunk per workgroup; cpw2, cpw4 built from the patch)
# parity, A/B 10:3 random, 20:3 1% loss, 20:3 m = 3
set -o pipefail
cd $GRAFT_REPO_ROOT
V=kcptube_amd/variants; O=gpurun_out/r4ad; mkdir -p $O
KFEC_LIB=$V/libkfec_cpw2.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_frame.py tests/test_gpu_pipeline.py -x -q --timeout 200 --timeout-method thread > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
L="kcptube_amd/libkfec.so $V/libkfec_cpw2.so $V/libkfec_cpw4.so"
AB_ERASE=random timeout -k 10 300 python tools/ab.py 3 $L -- 10 13 1400 1048576 > $O/ab_103.txt 2>&1 || { cat $O/ab_103.txt; exit 1; }
cat $O/ab_103.txt
AB_ERASE=iid:10000 timeout -k 10 300 python tools/ab.py 3 $L -- 20 23 1440 1048576 > $O/ab_203loss1.txt 2>&1 || { cat $O/ab_203loss1.txt; exit 1; }
cat $O/ab_203loss1.txt
timeout -k 10 300 python tools/ab.py 2 $L -- 20 23 1440 1048576 > $O/ab_203.txt 2>&1 || { cat $O/ab_203.txt; exit 1; }
cat $O/ab_203.txt
