#!/bin/bash
# Profile every bench config (kernel trace + PMC passes) and calibrate FETCH_SIZE on a known read.
set -o pipefail
bash tools/profile.sh r01_203 --steps 5 --warmup 1 --no-cpu || exit $?
bash tools/profile.sh r01_103dec --config 10:3dec --steps 5 --warmup 1 --no-cpu || exit $?
bash tools/profile.sh r01_20055 --config 200:55 --steps 2 --warmup 1 --no-cpu || exit $?
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/cal_fetch -o p -- ./tools/ceiling > gpurun_out/cal_fetch.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/cal_write -o p -- ./tools/ceiling > gpurun_out/cal_write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_wire -o kt -- python3 tools/bench_wire.py --steps 5 > gpurun_out/prof_wire.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_seal -o kt -- python3 tools/bench_seal.py --steps 3 > gpurun_out/prof_seal.log 2>&1 || exit $?
echo profiled
