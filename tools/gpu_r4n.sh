# round 4: Lagrange prep (200:55) and the listed syndrome kernel's prefetched list / headers (1% loss) -- parity,
# then A/B against the library before both changes
set -o pipefail
cd $GRAFT_REPO_ROOT
V=kcptube_amd/variants; O=gpurun_out/r4n; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_frame.py tests/test_gpu_pipeline.py -x -q --timeout 200 --timeout-method thread > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
AB_ERASE=iid:10000 timeout -k 10 300 python tools/ab.py 3 $V/libkfec_base.so kcptube_amd/libkfec.so -- 20 23 1440 1048576 > $O/ab_203loss1.txt 2>&1 || { cat $O/ab_203loss1.txt; exit 1; }
cat $O/ab_203loss1.txt
timeout -k 10 600 python tools/ab.py 2 $V/libkfec_base.so kcptube_amd/libkfec.so -- 200 255 1440 65536 > $O/ab_20055.txt 2>&1 || { cat $O/ab_20055.txt; exit 1; }
cat $O/ab_20055.txt
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o kt -- python3 tools/ab_one.py 200 255 1440 65536 > $O/kt.log 2>&1 || { tail $O/kt.log; exit 1; }
find $O/kt -name "kt_kernel_stats.csv" | head -1 | xargs cut -d, -f1-4 | head -6
