#!/bin/bash
# Seal/open evidence for profiles/: the bench line, a kernel trace of the same command, and the SQ counter
# passes of tools/gpu_seal_pmc.sh (base build only).  Outputs under gpurun_out/seal_prof/.
set -o pipefail
out=gpurun_out/seal_prof; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 200 python tools/bench_seal.py > $out/seal.json || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o kt -- python3 tools/bench_seal.py --steps 3 > $out/kt.log 2>&1 || exit 1
NOVAR=1 bash tools/gpu_seal_pmc.sh || exit 1
echo seal-prof-done
