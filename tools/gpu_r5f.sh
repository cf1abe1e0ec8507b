#!/bin/bash
# Round 5: sealed small-flush phases; 200:55 decode HBM traffic with factored records.
set -o pipefail
out=gpurun_out/r5f; mkdir -p $out
for mode in none chacha20; do KFEC_QUEUE_TRACE=1 PB_SEAL=$mode timeout -k 10 120 ./tools/pipeline_bench 20 23 1440 16 33 3 1 > $out/sealed_$mode.json 2> $out/sealed_$mode.err || exit 1; done
cut -c1-160 $out/sealed_*.json; cat $out/sealed_*.err
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for pmc in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $pmc --output-format csv -d $out/pmc_$pmc -o pmc -- python3 bench.py --config 200:55 --steps 2 --warmup 1 --no-cpu > $out/pmc_$pmc.log 2>&1 || exit 1
done
echo done
