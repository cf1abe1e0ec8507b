#!/bin/bash
# Round pass, part 2: every bench config under rocprofv3 (kernel trace + PMC passes), FETCH/WRITE calibration
# on known byte counts, wire / seal kernel traces.  Usage: tools/gpu_profile_all.sh <round tag, e.g. r02>
set -o pipefail
r=${1:-r02}
bash tools/profile.sh ${r}_203 --steps 5 --warmup 1 --no-cpu || exit $?
bash tools/profile.sh ${r}_103dec --config 10:3dec --steps 5 --warmup 1 --no-cpu || exit $?
bash tools/profile.sh ${r}_20055 --config 200:55 --steps 2 --warmup 1 --no-cpu || exit $?
bash tools/profile.sh ${r}_203loss1 --config 20:3loss1 --steps 5 --warmup 1 --no-cpu || exit $?
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/cal_fetch -o p -- ./tools/ceiling > gpurun_out/cal_fetch.log 2>&1 || exit $?
timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/cal_write -o p -- ./tools/ceiling > gpurun_out/cal_write.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_wire -o kt -- python3 tools/bench_wire.py --steps 5 > gpurun_out/prof_wire.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_seal -o kt -- python3 tools/bench_seal.py --steps 3 > gpurun_out/prof_seal.log 2>&1 || exit $?
echo profiled
