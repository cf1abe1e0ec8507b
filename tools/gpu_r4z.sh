# round 4: MAC / syndrome workgroup size (KFEC_MAC_BLOCK 128 / 512 vs 256): parity on each, A/B 10:3 random and 20:3
set -o pipefail
cd $GRAFT_REPO_ROOT
V=kcptube_amd/variants; O=gpurun_out/r4z; mkdir -p $O
for v in blk128 blk512; do
KFEC_LIB=$V/libkfec_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/parity_$v.log 2>&1 || { tail -30 $O/parity_$v.log; exit 1; }
tail -1 $O/parity_$v.log
done
L="kcptube_amd/libkfec.so $V/libkfec_blk128.so $V/libkfec_blk512.so"
AB_ERASE=random timeout -k 10 300 python tools/ab.py 3 $L -- 10 13 1400 1048576 > $O/ab_103.txt 2>&1 || { cat $O/ab_103.txt; exit 1; }
cat $O/ab_103.txt
timeout -k 10 300 python tools/ab.py 2 $L -- 20 23 1440 1048576 > $O/ab_203.txt 2>&1 || { cat $O/ab_203.txt; exit 1; }
cat $O/ab_203.txt
