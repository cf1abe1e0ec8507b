#!/bin/bash
# SQ counter passes over bench_aead.py (1M packets, one step): pass A = LDS / VALU work, pass B = where the
# wave cycles go (WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY = WAVE_CYCLES).  Summarise with
# tools/aead_pmc_table.py.  Outputs under gpurun_out/aead_pmc/.
set -o pipefail
out=gpurun_out/aead_pmc; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
A="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
B="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAVES"
for pass in A B; do
  timeout -s KILL 120 rocprofv3 --pmc ${!pass} --output-format csv -d $out/$pass -o p -- python3 tools/bench_aead.py --steps 1 --packets 1048576 --no-verify > $out/$pass.log 2>&1 || { tail $out/$pass.log; exit 1; }
done
echo pmc-done
