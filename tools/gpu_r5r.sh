#!/bin/bash
# Round 5: kernel durations of the small sealed flush (1 and 16 groups per flush) under rocprofv3 --kernel-trace.
set -o pipefail
out=gpurun_out/r5r; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for mode in none chacha20 aes_gcm; do for g in 1 16; do
  PB_SEAL=$mode timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt_${mode}_g$g -o kt -- ./tools/pipeline_bench 20 23 1440 $g 33 3 1 > $out/kt_${mode}_g$g.log 2>&1 || exit 1
done; done
for f in $out/kt_*/kt_kernel_stats.csv; do echo "== $f"; cut -d, -f1-4 $f | head -8; done
echo done
