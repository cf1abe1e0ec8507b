#!/bin/bash
# Profile one program on the GPU box (run through gpurun).  Writes under gpurun_out/prof_<tag>/.
#   pass 1: kernel trace + stats (per-kernel average duration)            (KT=0 skips it)
#   pass 2..: PMC counters, one group per pass (FETCH_SIZE and WRITE_SIZE cannot share a pass on gfx950)
# Usage: [PROG=tools/bench_seal.py] [PMC_SETS="A B C;D E"] [KFEC_LIB=...] tools/profile.sh <tag> [program args...]
#   PROG      the Python program profiled (default bench.py; args default to a short bench run)
#   PMC_SETS  ';'-separated counter groups, one rocprofv3 --pmc pass each (default: HBM bytes + SQ work / waits);
#             e.g. the seal / AEAD SQ passes of DESIGN §5b-5c:
#             PMC_SETS="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_LDS
#                       SQ_BUSY_CYCLES GRBM_GUI_ACTIVE;SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
#                       SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAVES"
#             KT=0 PROG=tools/bench_seal.py tools/profile.sh seal_base --steps 1 --packets 1048576
set -o pipefail
tag=${1:-r1}; shift
prog=${PROG:-bench.py}
args=${@:-"--steps 5 --warmup 1 --no-cpu"}
out=gpurun_out/prof_${tag}
mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
if [ "${KT:-1}" != 0 ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/kt -o kt -- python3 $prog $args > $out/kt.log 2>&1 || exit $?
fi
sets=${PMC_SETS:-"FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE;SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"}
IFS=';' read -ra groups <<< "$sets"
for pmc in "${groups[@]}"; do
  pmc=$(echo $pmc)  # (collapse the whitespace of a multi-line set)
  [ -z "$pmc" ] && continue
  name=$(echo $pmc | tr ' ' '_' | cut -c1-40)
  timeout -s KILL 300 rocprofv3 --pmc $pmc --output-format csv -d $out/pmc_$name -o pmc -- python3 $prog $args > $out/pmc_$name.log 2>&1 || exit $?
done
echo done
