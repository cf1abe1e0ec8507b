# round 4: 200:55 decode with the T-table entries -- parity, then interleaved A/B against the round-3 library
# (r3) and the same source with the old per-chunk expansion (tt0)
set -o pipefail
cd $GRAFT_REPO_ROOT
V=kcptube_amd/variants; O=gpurun_out/r4c; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
timeout -k 10 600 python tools/ab.py 2 $V/libkfec_r3.so $V/libkfec_tt0.so kcptube_amd/libkfec.so -- 200 255 1440 65536 > $O/ab_20055.txt 2>&1 || { cat $O/ab_20055.txt; exit 1; }
cat $O/ab_20055.txt
timeout -k 10 300 python tools/ab.py 2 $V/libkfec_r3.so kcptube_amd/libkfec.so -- 20 23 1440 1048576 > $O/ab_203.txt 2>&1 || { cat $O/ab_203.txt; exit 1; }
cat $O/ab_203.txt
