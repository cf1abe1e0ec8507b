# round 4: nontemporal shard loads (KFEC_NT_LOADS=1) vs default policy; linear-read ceiling with nt loads
set -o pipefail
cd $GRAFT_REPO_ROOT
V=kcptube_amd/variants; O=gpurun_out/r4g; mkdir -p $O
KFEC_LIB=$V/libkfec_ntl.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/parity_ntl.log 2>&1 || { tail -30 $O/parity_ntl.log; exit 1; }
tail -1 $O/parity_ntl.log
timeout -k 10 300 python tools/ab.py 3 kcptube_amd/libkfec.so $V/libkfec_ntl.so -- 20 23 1440 1048576 > $O/ab_203.txt 2>&1 || { cat $O/ab_203.txt; exit 1; }
cat $O/ab_203.txt
AB_ERASE=random timeout -k 10 300 python tools/ab.py 3 kcptube_amd/libkfec.so $V/libkfec_ntl.so -- 10 13 1400 1048576 > $O/ab_103.txt 2>&1 || { cat $O/ab_103.txt; exit 1; }
cat $O/ab_103.txt
timeout -k 10 200 tools/ceiling > $O/ceiling.txt 2>&1 || { cat $O/ceiling.txt; exit 1; }
head -8 $O/ceiling.txt
