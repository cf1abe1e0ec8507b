#!/bin/bash
# Profile the bench on the GPU box (run through gpurun).  Writes under gpurun_out/prof_<tag>/.
#   pass 1: kernel trace + stats (per-kernel average duration)
#   pass 2..: PMC counters, one group per pass (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950)
# Usage: tools/profile.sh <tag> [bench args...]
set -o pipefail
tag=${1:-r1}; shift
args=${@:-"--steps 5 --warmup 1 --no-cpu"}
out=gpurun_out/prof_${tag}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o kt -- python3 bench.py $args > $out/kt.log 2>&1 || exit $?
for pmc in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; do
  name=$(echo $pmc | tr ' ' '_' | cut -c1-40)
  timeout -k 10 300 rocprofv3 --pmc $pmc --output-format csv -d $out/pmc_$name -o pmc -- python3 bench.py $args > $out/pmc_$name.log 2>&1 || exit $?
done
echo done
