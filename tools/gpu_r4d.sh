# round 4: syndrome decode with 2 items per lane (K <= 12) -- parity, then interleaved A/B at 10:3 random 1-3 of 13
set -o pipefail
cd $GRAFT_REPO_ROOT
V=kcptube_amd/variants; O=gpurun_out/r4d; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $O/parity.log 2>&1 || { tail -30 $O/parity.log; exit 1; }
tail -1 $O/parity.log
KFEC_LIB=$V/libkfec_ipl3.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "batch or layout or digest" > $O/parity_ipl3.log 2>&1 || { tail -30 $O/parity_ipl3.log; exit 1; }
tail -1 $O/parity_ipl3.log
AB_ERASE=random timeout -k 10 600 python tools/ab.py 3 $V/libkfec_r3.so $V/libkfec_ipl1.so kcptube_amd/libkfec.so $V/libkfec_ipl3.so -- 10 13 1400 1048576 > $O/ab_103.txt 2>&1 || { cat $O/ab_103.txt; exit 1; }
cat $O/ab_103.txt
# the sealed queue (KFEC_TXQ_DEFER_DATA): throughput and the added send latency of the deferred data packets,
# at several flush sizes (groups per flush)
for mode in none chacha20; do
  for G in 16 256 4096 16384; do
    F=$(( G >= 4096 ? 4 : 32 ))
    PB_SEAL=$mode timeout -k 10 120 tools/pipeline_bench 20 23 1440 $G $F 3 1 >> $O/pipeline_sealed.jsonl 2>> $O/pipeline_sealed.err || { echo "pipeline_bench $mode $G failed"; cat $O/pipeline_sealed.err; exit 1; }
  done
done
timeout -k 10 120 tools/pipeline_bench 20 23 1440 16384 4 3 1 >> $O/pipeline_sealed.jsonl 2>> $O/pipeline_sealed.err
cat $O/pipeline_sealed.jsonl
