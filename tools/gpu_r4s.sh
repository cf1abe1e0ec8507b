# round 4: (1) encode for R <= 8 through enc_scalar_kernel (KFEC_ENC_SCALAR) vs mac_kernel (enc0);
# (2) syndrome-decode granules in flight for K <= 12 (KFEC_SYN_SMALLK_PD 5 / 6 vs 4)
set -o pipefail
cd $GRAFT_REPO_ROOT
V=kcptube_amd/variants; O=gpurun_out/r4s; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_frame.py tests/test_gpu_worker.py -x -q --timeout 200 --timeout-method thread > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
for v in spd5 spd6; do
KFEC_LIB=$V/libkfec_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/parity_$v.log 2>&1 || { tail -30 $O/parity_$v.log; exit 1; }
tail -1 $O/parity_$v.log
done
L="$V/libkfec_enc0.so kcptube_amd/libkfec.so"
timeout -k 10 300 python tools/ab.py 3 $L -- 20 23 1440 1048576 > $O/ab_enc203.txt 2>&1 || { cat $O/ab_enc203.txt; exit 1; }
cat $O/ab_enc203.txt
AB_ERASE=random timeout -k 10 300 python tools/ab.py 2 $L -- 10 13 1400 1048576 > $O/ab_enc103.txt 2>&1 || { cat $O/ab_enc103.txt; exit 1; }
cat $O/ab_enc103.txt
L="kcptube_amd/libkfec.so $V/libkfec_spd5.so $V/libkfec_spd6.so"
AB_ERASE=random timeout -k 10 300 python tools/ab.py 3 $L -- 10 13 1400 1048576 > $O/ab_103.txt 2>&1 || { cat $O/ab_103.txt; exit 1; }
cat $O/ab_103.txt
AB_ERASE=iid:10000 timeout -k 10 300 python tools/ab.py 2 $L -- 10 13 1400 1048576 > $O/ab_103loss1.txt 2>&1 || { cat $O/ab_103loss1.txt; exit 1; }
cat $O/ab_103loss1.txt
