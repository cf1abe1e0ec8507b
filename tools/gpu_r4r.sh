# round 4: granules in flight of the syndrome decode for K <= 12 (KFEC_SYN_SMALLK_PD 5 / 6 vs the default 4):
# parity on each variant, then A/B (fec=10:3 random 1-3 erasures, and 1% iid loss)
set -o pipefail
cd $GRAFT_REPO_ROOT
V=kcptube_amd/variants; O=gpurun_out/r4r; mkdir -p $O
L="kcptube_amd/libkfec.so $V/libkfec_spd5.so $V/libkfec_spd6.so"
for v in spd5 spd6; do
KFEC_LIB=$V/libkfec_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/parity_$v.log 2>&1 || { tail -30 $O/parity_$v.log; exit 1; }
tail -1 $O/parity_$v.log
done
AB_ERASE=random timeout -k 10 300 python tools/ab.py 3 $L -- 10 13 1400 1048576 > $O/ab_103.txt 2>&1 || { cat $O/ab_103.txt; exit 1; }
cat $O/ab_103.txt
AB_ERASE=iid:10000 timeout -k 10 300 python tools/ab.py 2 $L -- 10 13 1400 1048576 > $O/ab_103loss1.txt 2>&1 || { cat $O/ab_103loss1.txt; exit 1; }
cat $O/ab_103loss1.txt
