#!/bin/bash
# Resident-worker latency sweep: workgroups per worker (KFEC_WORKER_WGS) x doorbell spreading (KFEC_WORKER_POLL
# 0 relay / 1 direct), tools/latency_bench each; then the launch path (KFEC_WORKER=0).  One line per setting.
set -o pipefail
out=gpurun_out/worker_sweep; mkdir -p $out
for p in 0 1; do for wg in 2 4 8; do
  KFEC_WORKER_POLL=$p KFEC_WORKER_WGS=$wg timeout -k 5 60 ./tools/latency_bench > $out/lat_p${p}_w${wg}.json 2>&1 || { cat $out/lat_p${p}_w${wg}.json; exit 1; }
  echo "poll=$p wgs=$wg $(python3 -c "import json,sys; d=json.load(open('$out/lat_p${p}_w${wg}.json')); print({k: round(v,2) for k,v in d.items() if k.endswith('_us') and ('kfec_' in k or 'ping' in k)})")"
done; done
KFEC_WORKER=0 timeout -k 5 60 ./tools/latency_bench > $out/lat_launch.json 2>&1 || exit 1
echo "launch $(python3 -c "import json; d=json.load(open('$out/lat_launch.json')); print({k: round(v,2) for k,v in d.items() if k.endswith('_us') and 'kfec_' in k})")"
# small-K syndrome decode: granules in flight per lane (pd0 = the default PD = 4, pd6, pd10), 10:3 random 1-3 of 13
V=kcptube_amd/variants
KFEC_LIB=$V/libkfec_pd10.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "batch or sparse" --timeout 120 --timeout-method thread > $out/t_pd10.log 2>&1 || { tail -30 $out/t_pd10.log; exit 1; }
tail -1 $out/t_pd10.log
AB_ERASE=random timeout -k 10 400 python tools/ab.py 3 $V/libkfec_pd0.so $V/libkfec_pd6.so $V/libkfec_pd10.so -- 10 13 1400 1048576 > $out/ab_pd.txt 2>&1 || { cat $out/ab_pd.txt; exit 1; }
cat $out/ab_pd.txt
