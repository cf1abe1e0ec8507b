#!/bin/bash
# AEAD pass: GPU parity tests of the chacha20 / xchacha20 kernels, the throughput line (with the OpenSSL CPU
# leg), and a kernel trace of the same bench.  Outputs under gpurun_out/aead/.
set -o pipefail
out=gpurun_out/aead; mkdir -p $out
timeout -k 10 600 python -u -m pytest tests/test_gpu_aead.py -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $out/gtest.log 2>&1 || { tail -60 $out/gtest.log; exit 1; }
tail -3 $out/gtest.log
timeout -k 10 300 python -u tools/bench_aead.py --cpu-threads 16 > $out/bench.json 2> $out/bench.err || { tail -20 $out/bench.err; exit 1; }
cat $out/bench.json
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/prof -o kt -- python3 tools/bench_aead.py --steps 3 > $out/prof.log 2>&1 || { tail -20 $out/prof.log; exit 1; }
find $out/prof -name '*kernel_stats.csv' | head -1 | xargs cat | cut -c1-200 | head -12
echo aead-done
