# round 4: full GPU suite on the current library; 200:55 decode T-table A/B (tt1 shipped vs tt2: static T, one
# ds_read_u16 per row); the sealed pipeline (deferred data packets) throughput and send latency
set -o pipefail
cd $GRAFT_REPO_ROOT
V=kcptube_amd/variants; O=gpurun_out/r4e; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -3 $O/gpu_tests.log
KFEC_LIB=$V/libkfec_tt2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/parity_tt2.log 2>&1 || { tail -30 $O/parity_tt2.log; exit 1; }
tail -1 $O/parity_tt2.log
timeout -k 10 600 python tools/ab.py 3 kcptube_amd/libkfec.so $V/libkfec_tt2.so -- 200 255 1440 65536 > $O/ab_20055.txt 2>&1 || { cat $O/ab_20055.txt; exit 1; }
cat $O/ab_20055.txt
for mode in none chacha20; do
  for G in 16 256 4096 16384; do
    F=$(( G >= 4096 ? 5 : 33 ))
    PB_SEAL=$mode timeout -k 10 120 tools/pipeline_bench 20 23 1440 $G $F 3 1 >> $O/pipeline_sealed.jsonl 2>> $O/pipeline_sealed.err || { echo "pipeline_bench $mode $G failed"; cat $O/pipeline_sealed.err; exit 1; }
  done
done
timeout -k 10 120 tools/pipeline_bench 20 23 1440 16384 4 3 1 >> $O/pipeline_sealed.jsonl 2>> $O/pipeline_sealed.err
cat $O/pipeline_sealed.jsonl
