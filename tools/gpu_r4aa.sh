# round 4: syndrome-form decode on 16-byte granules (KFEC_SYN_VEC16; dense kernel 77 VGPRs) vs 32 (v32):
# parity through every decode user, A/B 10:3 random, 20:3 (m = 3), 20:3 at 1% loss, 30:36 random
set -o pipefail
cd $GRAFT_REPO_ROOT
V=kcptube_amd/variants; O=gpurun_out/r4aa; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_frame.py tests/test_gpu_pipeline.py tests/test_gpu_worker.py -x -q --timeout 200 --timeout-method thread > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
L="$V/libkfec_v32.so kcptube_amd/libkfec.so"
AB_ERASE=random timeout -k 10 300 python tools/ab.py 3 $L -- 10 13 1400 1048576 > $O/ab_103.txt 2>&1 || { cat $O/ab_103.txt; exit 1; }
cat $O/ab_103.txt
timeout -k 10 300 python tools/ab.py 2 $L -- 20 23 1440 1048576 > $O/ab_203.txt 2>&1 || { cat $O/ab_203.txt; exit 1; }
cat $O/ab_203.txt
AB_ERASE=iid:10000 timeout -k 10 300 python tools/ab.py 2 $L -- 20 23 1440 1048576 > $O/ab_203loss1.txt 2>&1 || { cat $O/ab_203loss1.txt; exit 1; }
cat $O/ab_203loss1.txt
AB_ERASE=random timeout -k 10 300 python tools/ab.py 2 $L -- 30 36 1440 262144 > $O/ab_306.txt 2>&1 || { cat $O/ab_306.txt; exit 1; }
cat $O/ab_306.txt
