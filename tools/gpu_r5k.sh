#!/bin/bash
# Round 5: T-table decode offsets read per row straight into the table address (KFEC_DEC_OFS16; now dec_expand_fac, KFEC_DEC_EXPAND2) -- parity and
# an interleaved 200:55 A/B against the previous form, then the 200:55 decode's HBM traffic.
set -o pipefail
out=gpurun_out/r5k; mkdir -p $out; V=kcptube_amd/variants
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > $out/t1.log 2>&1 || { tail -40 $out/t1.log; exit 1; }
tail -1 $out/t1.log
AB_ITERS=4 timeout -k 10 600 python tools/ab.py 3 kcptube_amd/libkfec.so $V/libkfec_exp1.so -- 200 255 1440 262144 > $out/ab_20055.txt || exit 1
cat $out/ab_20055.txt
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for pmc in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $pmc --output-format csv -d $out/pmc_$pmc -o pmc -- python3 bench.py --config 200:55 --steps 2 --warmup 1 --no-cpu > $out/pmc_$pmc.log 2>&1 || exit 1
done
echo done
