#!/bin/bash
# One SQ counter pass over bench_aead for the shipped build and each variant in kcptube_amd/variants.
set -o pipefail
out=gpurun_out/aead_pmc; mkdir -p $out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for v in base $(cd kcptube_amd/variants 2>/dev/null && ls libkfec_aead_*.so 2>/dev/null | sed 's/libkfec_//; s/\.so//'); do
  lib=""; [ "$v" != base ] && lib=kcptube_amd/variants/libkfec_$v.so
  KFEC_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE --output-format csv -d $out/$v -o p -- python3 tools/bench_aead.py --steps 1 --packets 1048576 --no-verify > $out/$v.log 2>&1 || { tail $out/$v.log; exit 1; }
done
echo pmc-done
