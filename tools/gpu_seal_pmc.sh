#!/bin/bash
# SQ counter passes over bench_seal.py for the shipped build and each kcptube_amd/variants/libkfec_seal_*.so:
# pass a = LDS / VALU work, pass b = where the wave cycles go (WAIT_ANY + WAIT_INST_ANY + ACTIVE_INST_ANY
# = WAVE_CYCLES, MI355X_MICROARCH.md "SQ")
set -o pipefail
out=gpurun_out/seal_pmc; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
A="SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
B="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_WAVES"
for v in base $([ -n "$NOVAR" ] || (cd kcptube_amd/variants && ls libkfec_seal_*.so 2>/dev/null | sed "s/libkfec_//; s/\.so//")); do
  lib=""; [ "$v" != base ] && lib=kcptube_amd/variants/libkfec_$v.so
  for pass in A B; do
    KFEC_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc ${!pass} --output-format csv -d $out/${v}_$pass -o p -- python3 tools/bench_seal.py --steps 1 --packets 1048576 > $out/${v}_$pass.log 2>&1 || { tail $out/${v}_$pass.log; exit 1; }
  done
done
echo pmc-done
