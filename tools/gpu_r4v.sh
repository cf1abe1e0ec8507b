# round 4: syn_final re-extracts the selectors per output row (KFEC_SYN_FINAL_RECOMP): syn_kernel<32,3> 110 -> 93
# VGPRs (5 waves per SIMD), <32,8> 255 -> 168.  Parity on the shipped build, A/B against recomp0.
set -o pipefail
cd $GRAFT_REPO_ROOT
V=kcptube_amd/variants; O=gpurun_out/r4v; mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_frame.py -x -q --timeout 200 --timeout-method thread > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
L="$V/libkfec_recomp0.so kcptube_amd/libkfec.so"
AB_ERASE=random timeout -k 10 300 python tools/ab.py 3 $L -- 10 13 1400 1048576 > $O/ab_103.txt 2>&1 || { cat $O/ab_103.txt; exit 1; }
cat $O/ab_103.txt
timeout -k 10 300 python tools/ab.py 3 $L -- 20 23 1440 1048576 > $O/ab_203.txt 2>&1 || { cat $O/ab_203.txt; exit 1; }
cat $O/ab_203.txt
AB_ERASE=random timeout -k 10 300 python tools/ab.py 2 $L -- 30 36 1440 262144 > $O/ab_306.txt 2>&1 || { cat $O/ab_306.txt; exit 1; }
cat $O/ab_306.txt
